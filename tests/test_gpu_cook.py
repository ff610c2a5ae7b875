"""GPU parity for the batched packet cook / de_cook kernels.

Compares librsmi's HIP path with the oracle (oracle/cook_oracle.c, itself
pinned to the reference packet.cpp by tests/test_cook_oracle.py) and with the
reference's own vectors (tests/golden/cook_vectors.npz).  Bit-exact: every byte
of every packet slot, output lengths and de_cook status.
"""
import numpy as np
import pytest

from oracle.cpu import (NO_CHECKSUM, NO_OBSCURE, NO_XOR, cook_ivs, cook_payloads, device_ivs,
                        recover_iv)

pytestmark = pytest.mark.gpu

KEYS = [b"", b"k", b"passwd123", bytes(range(1, 200))]


def _tensors(gpu, buf, lens, iv=None, ivl=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(buf)).to(gpu)
    ln = torch.from_numpy(np.ascontiguousarray(lens, np.int32)).to(gpu)
    out = [t, ln]
    if iv is not None:
        out += [torch.from_numpy(np.ascontiguousarray(iv)).to(gpu),
                torch.from_numpy(np.ascontiguousarray(ivl, np.uint8)).to(gpu)]
    return out


def _oracle_cook(cook_oracle, buf, lens, iv, ivl, key, flags):
    ref = buf.copy()
    out = cook_oracle.cook_batch(ref, ref.shape[1], lens, iv, ivl, key, flags)
    return ref, out


def test_golden_vectors_cook_decook(gpu, cook_vectors):
    import torch
    from udpspeeder_amd.cook import CookContext
    z = cook_vectors
    groups = {}
    for i in range(z.n):
        c = z.case(i)
        groups.setdefault((c["key"], c["flags"]), []).append(c)
    for (key, flags), cases in groups.items():
        ctx = CookContext(key, flags)
        stride = 1344
        npk = len(cases)
        buf = np.zeros((npk, stride), np.uint8)
        lens = np.array([len(c["plain"]) for c in cases], np.int32)
        iv = np.zeros((npk, 32), np.uint8)
        ivl = np.zeros(npk, np.uint8)
        for j, c in enumerate(cases):
            buf[j, :lens[j]] = np.frombuffer(c["plain"], np.uint8)
            v, vl = recover_iv(c["cooked"], lens[j], key, flags)
            iv[j, :vl] = np.frombuffer(v, np.uint8)
            ivl[j] = vl
        t, ln, tiv, tivl = _tensors(gpu, buf, lens, iv, ivl)
        out = ctx.cook(t, ln, cap=stride, iv=tiv, iv_len=tivl).cpu().numpy()
        got = t.cpu().numpy()
        for j, c in enumerate(cases):
            assert out[j] == len(c["cooked"]), (key, flags, j)
            assert got[j, :out[j]].tobytes() == c["cooked"], (key, flags, lens[j])
        # de_cook the reference's cooked bytes
        cb = np.zeros((npk, stride), np.uint8)
        clen = np.array([len(c["cooked"]) for c in cases], np.int32)
        for j, c in enumerate(cases):
            cb[j, :clen[j]] = np.frombuffer(c["cooked"], np.uint8)
        t, ln = _tensors(gpu, cb, clen)
        back = ctx.decook(t, ln, cap=stride).cpu().numpy()
        got = t.cpu().numpy()
        for j, c in enumerate(cases):
            assert back[j] == lens[j]
            assert got[j, :lens[j]].tobytes() == c["plain"]
        # corrupted packets: status and the buffer the reference leaves behind
        bad = [c for c in cases if c["bad_in"]]
        if bad:
            bb = np.zeros((len(bad), stride), np.uint8)
            blen = np.array([len(c["bad_in"]) for c in bad], np.int32)
            for j, c in enumerate(bad):
                bb[j, :blen[j]] = np.frombuffer(c["bad_in"], np.uint8)
            t, ln = _tensors(gpu, bb, blen)
            st = ctx.decook(t, ln, cap=stride).cpu().numpy()
            got = t.cpu().numpy()
            for j, c in enumerate(bad):
                assert (st[j] >= 0) == (c["bad_status"] == 0), (key, flags, j)
                assert got[j, :blen[j]].tobytes() == c["bad_out"]
                if st[j] >= 0:
                    assert st[j] == c["bad_len"]
        ctx.close()
        torch.cuda.synchronize()


@pytest.mark.parametrize("flags", range(8))
@pytest.mark.parametrize("key", KEYS)
def test_random_batch_vs_oracle(gpu, cook_oracle, key, flags):
    from udpspeeder_amd.cook import CookContext
    npk, stride = 777, 3136
    rng = np.random.default_rng(flags * 31 + len(key))
    lens = rng.integers(0, 3020, npk).astype(np.int32)
    lens[:40] = np.arange(40)                       # every short length
    lens[40:60] = 1536 + np.arange(-10, 10)         # round boundary
    buf = cook_payloads(0xC0DE + flags, 0, npk, lens, stride)
    buf[:, -64:] = 0xA5                              # sentinel beyond every packet
    iv, ivl = cook_ivs(0xC0DE, 0, npk)
    ivl[:33] = np.arange(33)                        # iv_len 0..32
    want, wout = _oracle_cook(cook_oracle, buf, lens, iv, ivl, key, flags)
    ctx = CookContext(key, flags)
    t, ln, tiv, tivl = _tensors(gpu, buf, lens, iv, ivl)
    out = ctx.cook(t, ln, cap=stride - 64, iv=tiv, iv_len=tivl).cpu().numpy()
    assert (out == wout).all()
    got = t.cpu().numpy()
    assert (got == want).all()                       # whole slots, incl. untouched bytes
    # and back
    back = ctx.decook(t, _tensors(gpu, buf, out)[1], cap=stride - 64).cpu().numpy()
    assert (back == lens).all()
    ref2 = want.copy()
    wback = cook_oracle.decook_batch(ref2, stride, wout, key, flags)
    assert (wback == back).all()
    assert (t.cpu().numpy() == ref2).all()


def test_device_drawn_ivs(gpu, cook_oracle):
    from udpspeeder_amd.cook import CookContext
    npk, stride, seed = 1000, 1344, 0xABCDEF
    lens = (np.arange(npk) * 7 % 1290).astype(np.int32)
    buf = cook_payloads(1, 0, npk, lens, stride)
    iv, ivl = device_ivs(seed, 0, npk)
    assert ivl.min() >= 4 and ivl.max() <= 32
    want, wout = _oracle_cook(cook_oracle, buf, lens, iv, ivl, b"key", 0)
    ctx = CookContext(b"key", 0)
    t, ln = _tensors(gpu, buf, lens)
    out = ctx.cook(t, ln, cap=stride, seed=seed).cpu().numpy()
    assert (out == wout).all()
    assert (t.cpu().numpy() == want).all()


@pytest.mark.parametrize("flags", [0, NO_CHECKSUM, NO_OBSCURE, NO_XOR])
def test_corruption_vs_oracle(gpu, cook_oracle, flags):
    """Flip bits / truncate / forge iv_len bytes up to 255: status and buffer."""
    from udpspeeder_amd.cook import CookContext
    key = b"corrupt-key"
    npk, stride = 2000, 1600
    rng = np.random.default_rng(99 + flags)
    lens = rng.integers(0, 1500, npk).astype(np.int32)
    buf = cook_payloads(5, 0, npk, lens, stride)
    iv, ivl = cook_ivs(5, 0, npk)
    cooked, clen = _oracle_cook(cook_oracle, buf, lens, iv, ivl, key, flags)
    for i in range(npk):
        mode = i % 4
        if mode == 1 and clen[i]:
            cooked[i, rng.integers(0, clen[i])] ^= 1 << int(rng.integers(0, 8))
        elif mode == 2 and clen[i]:
            clen[i] = rng.integers(0, clen[i])
        elif mode == 3 and clen[i]:   # forge the trailing iv_len byte (after the key)
            kb = key[(clen[i] - 1) % len(key)] if not flags & NO_XOR else 0
            cooked[i, clen[i] - 1] = int(rng.integers(0, 256)) ^ kb
    want = cooked.copy()
    wst = cook_oracle.decook_batch(want, stride, clen, key, flags)
    ctx = CookContext(key, flags)
    t, ln = _tensors(gpu, cooked, clen)
    st = ctx.decook(t, ln, cap=stride).cpu().numpy()
    assert (st == wst).all()
    assert (t.cpu().numpy() == want).all()
    assert (wst >= 0).sum() > npk // 8 and (wst < 0).sum() > 0
    if not flags & NO_CHECKSUM:                  # the crc catches flips and truncations
        assert (wst < 0).sum() > npk // 4


def test_offsets_and_alignment(gpu, cook_oracle):
    """Packets at explicit offsets with 4-, 8- and 12-byte misalignment (the
    framed FEC packet starts 8 bytes before a 16-aligned shard)."""
    import torch
    from udpspeeder_amd.cook import CookContext
    npk, slot = 300, 1408
    lens = ((np.arange(npk) * 53) % 1300).astype(np.int32)
    offs = np.arange(npk, dtype=np.int64) * slot + 4 * (np.arange(npk) % 4)
    plain = cook_payloads(11, 0, npk, lens, slot - 16)
    flat = np.full(npk * slot, 0x5A, np.uint8)
    for i in range(npk):
        flat[offs[i]:offs[i] + slot - 16] = plain[i]
    iv, ivl = cook_ivs(11, 0, npk)
    ctx = CookContext(b"align", 0)
    t = torch.from_numpy(flat.copy()).to(gpu)
    ln = torch.from_numpy(lens).to(gpu)
    to = torch.from_numpy(offs).to(gpu)
    out = ctx.cook(t, ln, cap=slot - 16, offsets=to, iv=torch.from_numpy(iv).to(gpu),
                   iv_len=torch.from_numpy(ivl).to(gpu)).cpu().numpy()
    got = t.cpu().numpy()
    want = plain.copy()
    wout = cook_oracle.cook_batch(want, slot - 16, lens, iv, ivl, b"align", 0)
    assert (out == wout).all()
    for i in range(npk):
        assert (got[offs[i]:offs[i] + slot - 16] == want[i]).all(), i
    # bytes outside every packet's slot are untouched
    mask = np.ones(npk * slot, bool)
    for i in range(npk):
        mask[offs[i]:offs[i] + slot - 16] = False
    assert (got[mask] == 0x5A).all()


def test_rejections(gpu):
    from udpspeeder_amd.cook import CookContext
    ctx = CookContext(b"x", 0)
    stride = 128
    lens = np.array([100, 80, 91, -1, 0], np.int32)   # 100+37 > 128: reject; 91+37=128 ok
    iv = np.zeros((5, 32), np.uint8)
    ivl = np.array([32, 40, 32, 4, 4], np.uint8)       # 40 > IV_MAX: reject
    buf = np.arange(5 * stride, dtype=np.uint32).astype(np.uint8).reshape(5, stride)
    t, ln, tiv, tivl = _tensors(gpu, buf, lens, iv, ivl)
    out = ctx.cook(t, ln, cap=stride, iv=tiv, iv_len=tivl).cpu().numpy()
    assert list(out) == [-1, -1, 91 + 37, -1, 0 + 4 + 4 + 1]
    got = t.cpu().numpy()
    for i in (0, 1, 3):
        assert (got[i] == buf[i]).all()
    with pytest.raises(ValueError):
        ctx.cook(t, ln, cap=stride, iv=tiv)


def test_long_packets(gpu, cook_oracle):
    """Up to RSMI_COOK_MAX_LEN: many rounds, z digits all exercised."""
    from udpspeeder_amd.cook import CookContext
    lens = np.array([65535 - 37, 65535, 40000, 4095, 4096, 4097, 3071, 3072, 3073, 6144], np.int32)
    stride = 65536 + 64
    buf = cook_payloads(77, 0, len(lens), lens, stride)
    iv, ivl = cook_ivs(77, 0, len(lens))
    want, wout = _oracle_cook(cook_oracle, buf, lens, iv, ivl, b"long key", 0)
    ctx = CookContext(b"long key", 0)
    t, ln, tiv, tivl = _tensors(gpu, buf, lens, iv, ivl)
    out = ctx.cook(t, ln, cap=stride, iv=tiv, iv_len=tivl).cpu().numpy()
    assert list(out) == list(wout)
    assert (t.cpu().numpy() == want).all()
    back = ctx.decook(t, _tensors(gpu, buf, out)[1], cap=stride).cpu().numpy()
    # 65535 + 37 > RSMI_COOK_MAX_LEN: that cooked packet is rejected by de_cook's bound
    assert back[0] == lens[0] and back[1] == -1 and (back[2:] == lens[2:]).all()


def test_host_forms_and_reference_mirror(gpu, cook_oracle):
    import udpspeeder_amd.cook as ck
    ctx = ck.CookContext(b"host", NO_OBSCURE)
    npk, stride = 50, 512
    lens = (np.arange(npk) * 9).astype(np.int32)
    buf = cook_payloads(3, 0, npk, lens, stride)
    want = buf.copy()
    wout = cook_oracle.cook_batch(want, stride, lens, np.zeros((npk, 32), np.uint8),
                                  np.zeros(npk, np.uint8), b"host", NO_OBSCURE)
    out = ctx.cook_host(buf, lens)
    assert (out == wout).all() and (buf == want).all()
    back = ctx.decook_host(buf, out)
    assert (back == lens).all()
    # packet.h-style per-packet calls with the reference's globals
    ck.key_string, ck.disable_checksum, ck.disable_obscure, ck.disable_xor = b"mirror", 0, 0, 0
    data = bytearray(b"hello udpspeeder" + bytes(64))
    n = ck.do_cook(data, 16)
    assert 16 + 4 + 4 + 1 <= n <= 16 + 4 + 32 + 1
    rc, buf2, ln2 = cook_oracle.de_cook(bytes(data[:n]), b"mirror", 0)
    assert rc == 0 and buf2[:ln2] == b"hello udpspeeder"
    rc, ln = ck.de_cook(data, n)
    assert rc == 0 and ln == 16 and bytes(data[:16]) == b"hello udpspeeder"
    data = bytearray(b"hello udpspeeder" + bytes(64))
    n = ck.do_cook(data, 16)
    data[3] ^= 1                       # a payload bit: the crc check fails
    assert ck.de_cook(data, n)[0] == -1
    bad = bytearray(b"\x00\x01\x02")
    assert ck.de_cook(bad, 3)[0] == -1


def test_full_size_round_trip(gpu):
    """All 30 framed packets of 65,536 RS(20,10) groups (1258 B each): cook with
    device IVs, de_cook, compare (size-independent property)."""
    import torch
    from udpspeeder_amd.cook import CookContext
    npk, ln_, stride = 65536 * 30 // 8, 1258, 1312
    base = torch.randint(0, 256, (npk, stride), dtype=torch.uint8, device=gpu)
    orig = base.clone()
    lens = torch.full((npk,), ln_, dtype=torch.int32, device=gpu)
    ctx = CookContext(b"full-size", 0)
    out = ctx.cook(base, lens, cap=stride, seed=42)
    assert int(out.min()) >= ln_ + 9 and int(out.max()) <= ln_ + 37
    assert not torch.equal(base[:, :ln_], orig[:, :ln_])
    back = ctx.decook(base, out, cap=stride)
    assert bool((back == ln_).all())
    assert torch.equal(base[:, :ln_], orig[:, :ln_])


@pytest.mark.parametrize("host", [False, True])
def test_out_of_place_and_pinned_host(gpu, cook_oracle, host):
    """rsmi_cook_to writes every cooked packet at the same offset of another
    buffer -- device memory, or pinned host memory the kernel's stores reach
    over PCIe (the send side's cook + D2H in one pass) -- and leaves the source
    untouched; rsmi_decook_to reads a pinned host batch over PCIe (the receive
    side's H2D + de_cook in one pass).  Bytes and lengths equal the oracle's
    in-place transforms."""
    import torch
    from udpspeeder_amd.cook import CookContext
    rng = np.random.default_rng(41 + host)
    npk, stride, key = 300, 1344, b"passwd123"
    lens = rng.integers(0, 1300, npk).astype(np.int32)
    lens[:4] = [0, 1, 15, 16]
    buf = rng.integers(0, 256, (npk, stride), dtype=np.uint8)
    iv, ivl = cook_ivs(7, 0, npk)
    ref, out_ref = _oracle_cook(cook_oracle, buf, lens, iv, ivl, key, 0)
    t, ln, tiv, tivl = _tensors(gpu, buf, lens, iv, ivl)
    ctx = CookContext(key)
    dst = torch.zeros(npk * stride, dtype=torch.uint8)
    dst = dst.pin_memory() if host else dst.to(gpu)
    ol = ctx.cook_to(t, ln, dst, cap=stride, stride=stride, iv=tiv, iv_len=tivl)
    torch.cuda.synchronize()
    ol = ol.cpu().numpy()
    assert (ol == out_ref).all()
    got = dst.cpu().numpy().reshape(npk, stride)
    for j in range(npk):
        assert (got[j, :ol[j]] == ref[j, :ol[j]]).all(), j
    assert (t.cpu().numpy() == buf).all()  # the source is read only
    # de_cook from pinned host memory into the device
    src = torch.from_numpy(ref.reshape(-1).copy()).pin_memory()
    dec = torch.zeros(npk * stride, dtype=torch.uint8, device=gpu)
    ln2 = torch.from_numpy(out_ref.astype(np.int32)).to(gpu)
    ol2 = ctx.decook_to(src, ln2, dec, cap=stride, stride=stride)
    torch.cuda.synchronize()
    assert (ol2.cpu().numpy() == lens).all()
    back = dec.cpu().numpy().reshape(npk, stride)
    for j in range(npk):
        assert (back[j, :lens[j]] == buf[j, :lens[j]]).all(), j


@pytest.mark.gpu
def test_decook_mirror_to_pinned_host(gpu, cook_oracle):
    """rsmi_decook_mirror: de_cook in place on the device and the same bytes
    into a pinned host buffer (the tunnel's receive side), including packets
    whose de_cook fails (a flipped byte): the host copy equals the device's
    in-place result wherever de_cook wrote, and the payloads equal the input."""
    import torch
    from udpspeeder_amd.cook import CookContext
    rng = np.random.default_rng(77)
    npk, stride, key = 257, 1408, b"mirror-key"
    lens = rng.integers(0, 1340, npk).astype(np.int32)
    lens[:3] = [0, 1, 16]
    buf = rng.integers(0, 256, (npk, stride), dtype=np.uint8)
    iv, ivl = cook_ivs(9, 0, npk)
    ref, out_ref = _oracle_cook(cook_oracle, buf, lens, iv, ivl, key, 0)
    bad = rng.choice(npk, 20, replace=False)
    for j in bad:
        ref[j, rng.integers(0, out_ref[j])] ^= 0x40
    ctx = CookContext(key)
    d = torch.from_numpy(ref.reshape(-1).copy()).to(gpu)
    host = torch.full((npk * stride,), 0x5A, dtype=torch.uint8).pin_memory()
    ln = torch.from_numpy(out_ref.astype(np.int32)).to(gpu)
    ol = ctx.decook_mirror(d, ln, host, cap=stride, stride=stride).cpu().numpy()
    torch.cuda.synchronize()
    dev = d.cpu().numpy().reshape(npk, stride)
    h = host.numpy().reshape(npk, stride)
    for j in range(npk):
        e = (int(out_ref[j]) + 15) // 16 * 16
        assert (h[j, :e] == dev[j, :e]).all(), j
        assert (h[j, e:] == 0x5A).all(), j  # nothing past the packet's pieces
        if j in bad:
            continue
        assert ol[j] == lens[j], j
        assert (h[j, :lens[j]] == buf[j, :lens[j]]).all(), j
    rc = [cook_oracle.de_cook(ref[j, :out_ref[j]].tobytes(), key)[0] for j in bad]
    assert [int(ol[j]) < 0 for j in bad] == [r != 0 for r in rc]

