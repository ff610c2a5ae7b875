"""Several GPUs behind the host-memory entry points (SURVEY.md §8e,
include/rsmi.h rsmi_set_devices): the range split on the CPU, and on the GPU
the split pipelines bit-exact against the single-device path and the oracle.
On the 1-GPU box the device list [0, 0] (and [0, 0, 0]) runs two (three)
workers with their own streams and buffers on one device: the same partition,
threads and joins as eight devices."""
import numpy as np
import pytest

import udpspeeder_amd as u
from udpspeeder_amd import shard


@pytest.mark.parametrize("n,parts", [(0, 1), (1, 3), (7, 2), (65536, 8), (1 << 20, 8), (1000, 7)])
def test_split_ranges_uniform_matches_strong_range(n, parts):
    got = u.rs.split_ranges(n, parts)
    assert got == [shard.strong_range(r, parts, n) for r in range(parts)]


@pytest.mark.parametrize("seed,n,parts", [(1, 1000, 2), (2, 65536, 8), (3, 5, 8), (4, 300, 3)])
def test_split_ranges_cost_matches_balanced_ranges(seed, n, parts):
    """Cost-balanced cuts are shard.balanced_ranges' (C3: cost = (k+m)*len)."""
    rng = np.random.default_rng(seed)
    cost = rng.integers(0, 30 * 1250, n)
    assert u.rs.split_ranges(n, parts, cost) == shard.balanced_ranges(cost, parts)


def test_split_ranges_and_set_devices_reject_bad_args():
    from udpspeeder_amd._lib import RsmiError
    with pytest.raises(RsmiError):
        u.rs.split_ranges(10, 0)
    with pytest.raises(RsmiError):
        u.rs.split_ranges(3, 2, [1, -1, 2])
    assert u.lib().rsmi_set_devices(None, -1) != 0
    assert u.lib().rsmi_set_devices(None, 2) != 0
    assert u.rs.get_devices() == []


@pytest.mark.gpu
@pytest.mark.parametrize("devs", [[0], [0, 0], [0, 0, 0]])
def test_multidev_encode_decode_pinned(gpu, oracle, devs):
    """encode_pinned / decode_pinned over the device list: parity equal to the
    oracle's, the decode's rebuilt rows and statuses equal the single-device
    call's, for pinned (zero-copy decode) and pageable (staged) host memory."""
    import torch
    k, n, ln, S, G = 20, 30, 1250, 1280, 3001  # G not a multiple of the device count
    rng = np.random.default_rng(55)
    data = rng.integers(0, 256, (G, k, S), dtype=np.uint8)
    try:
        u.rs.set_devices(devs)
        assert u.rs.get_devices() == devs
        for pinned in (True, False):
            d = torch.from_numpy(data.copy())
            par = torch.zeros((G, n - k, S), dtype=torch.uint8)
            if pinned:
                d, par = d.pin_memory(), par.pin_memory()
            u.rs.encode_pinned(d, par, k, n, ln, chunk_groups=512)
            ref = np.zeros((G, n, S), np.uint8)
            ref[:, :k] = data
            oracle.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G)
            assert np.array_equal(par.numpy()[:, :, :ln], ref[:, k:, :ln]), pinned
            # decode: the whole codeword, 5 random erasures per group, data slots wiped
            full = np.concatenate([data, par.numpy()], axis=1)
            pres = np.ones((G, n), np.uint8)
            for g in range(G):
                pres[g, rng.choice(n, 5, replace=False)] = 0
            h = torch.from_numpy(full.copy())
            h[torch.from_numpy(pres == 0)] = 0xA5
            if pinned:
                h = h.pin_memory()
            st = u.rs.decode_pinned(h, pres, k, n, ln, chunk_groups=700)
            assert (st == 0).all()
            assert np.array_equal(h.numpy()[:, :k, :ln], data[:, :, :ln]), pinned
            path = u.lib().rsmi_last_decode_pinned_path()
            assert path == (1 if pinned else 2), path
    finally:
        u.rs.set_devices([])
    assert u.rs.get_devices() == []


@pytest.mark.gpu
def test_multidev_error_names_the_device(gpu):
    """An invalid device list is rejected and leaves the pool as it was; the
    pool then still runs (an all-zero batch encodes to zero parity)."""
    from udpspeeder_amd._lib import RsmiError
    import torch
    try:
        u.rs.set_devices([0, 0])
        with pytest.raises(RsmiError, match="out of range"):
            u.rs.set_devices([0, 99])
        assert u.rs.get_devices() == [0, 0]  # a rejected list leaves the pool as it was
        d = torch.zeros((64, 4, 256), dtype=torch.uint8)
        p = torch.zeros((64, 2, 256), dtype=torch.uint8)
        u.rs.encode_pinned(d, p, 4, 6, 200)
        assert int(p.sum()) == 0
    finally:
        u.rs.set_devices([])
