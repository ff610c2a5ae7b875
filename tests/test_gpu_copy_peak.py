"""rsmi_copy_peak (bench.py's measured copy line): every variant copies exactly
the bytes asked for, tails of a partial block included, and rejects sizes and
pointers it does not handle."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("nbytes", [16, 4096, 16 * 256 * 4 + 48, 16 * 256 * 8 * 3 - 16, 5 << 20])
def test_copy_peak_exact(gpu, variant, nbytes):
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd._lib import check
    g = torch.Generator(device="cpu").manual_seed(nbytes + variant)
    src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, generator=g).to(gpu)
    dst = torch.full((nbytes + 64,), 0xA5, dtype=torch.uint8, device=gpu)
    check(u.lib().rsmi_copy_peak(dst.data_ptr(), src.data_ptr(), nbytes, variant, None), "rsmi_copy_peak")
    torch.cuda.synchronize()
    assert torch.equal(dst[:nbytes], src[:nbytes])
    assert bool((dst[nbytes:] == 0xA5).all())  # nothing past the end


def test_copy_peak_rejects(gpu):
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd._lib import RSMI_ERR_INVALID
    a = torch.zeros(4096, dtype=torch.uint8, device=gpu)
    L = u.lib()
    assert L.rsmi_copy_peak(a.data_ptr(), a.data_ptr() + 2048, 20, 0, None) == RSMI_ERR_INVALID
    assert L.rsmi_copy_peak(a.data_ptr() + 8, a.data_ptr() + 2048, 32, 0, None) == RSMI_ERR_INVALID
    assert L.rsmi_copy_peak(a.data_ptr(), a.data_ptr() + 2048, 32, 4, None) == RSMI_ERR_INVALID
    assert L.rsmi_copy_peak(a.data_ptr(), a.data_ptr() + 2048, 0, 0, None) == 0


@pytest.mark.parametrize("variant,R,W", [(5, 4, 2), (6, 6, 1), (4, 4, 0)])
def test_mix_peak_writes_its_share(gpu, variant, R, W):
    """The read:write mixes write, per thread, the XOR of its words u = w mod W
    (variant 4 writes nothing)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd._lib import check
    nbytes = 16 * 256 * 24 * 3
    g = torch.Generator(device="cpu").manual_seed(variant)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).to(gpu)
    dst = torch.zeros(nbytes, dtype=torch.uint8, device=gpu)
    check(u.lib().rsmi_copy_peak(dst.data_ptr(), src.data_ptr(), nbytes, variant, None), "rsmi_copy_peak")
    torch.cuda.synchronize()
    if W == 0:
        assert int(dst.count_nonzero()) == 0
        return
    words = src.view(torch.int32).view(-1, R, 64, 4)  # per wave: R instructions of 64 lanes
    exp = torch.zeros((words.shape[0], W, 64, 4), dtype=torch.int32, device=gpu)
    for uu in range(R):
        exp[:, uu % W] ^= words[:, uu]
    got = dst.view(torch.int32)[:exp.numel()].view(exp.shape)
    assert torch.equal(got, exp)
    assert int(dst[exp.numel() * 4:].count_nonzero()) == 0
