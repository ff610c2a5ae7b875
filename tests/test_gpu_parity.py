"""GPU parity: the HIP path (through librsmi.so's C ABI) against the reference's
golden fixtures and the C oracle, bit-exact.  Full-size C1/C2/C3 batches are
checked against sha256 digests produced by the reference itself."""
import hashlib
import os

import numpy as np
import pytest

from oracle.cpu import DATA_SEED, ERASE_SEED, RAGGED_SEED, group_data
from oracle.gen_golden import ENCODE_CASES, C3_STR

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stride_for(ln):
    return max(16, (ln + 15) // 16 * 16)


def pad_end(ln, stride):
    """rsmi.h slot-padding rule: kernels may touch [len, pad_end) only."""
    return min(stride, (ln + 127) // 128 * 128)


def upload(buf, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(buf)).to(device)


def _decode_cases():
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "decode_small.npz"))
    return sorted({k.split("__")[0] for k in d.files})


# ---------------------------------------------------------------- synthetic data
def test_fill_matches_stream_definition(gpu):
    import torch
    import udpspeeder_amd as u
    for (k, ln, G, g0) in [(20, 1250, 7, 0), (3, 17, 5, 11), (1, 1, 3, 2), (13, 257, 4, 100)]:
        S = stride_for(ln)
        t = torch.zeros((G, k + 2, S), dtype=torch.uint8, device=gpu)
        u.fill_data(t, k, ln, DATA_SEED, g0=g0)
        got = t.cpu().numpy()
        assert (got[:, :k, :ln] == group_data(DATA_SEED, g0, G, k, ln)).all()
        assert (got[:, k:] == 0).all()


# ---------------------------------------------------------------- encode
@pytest.mark.parametrize("case", ENCODE_CASES)
def test_encode_small_golden(gpu, golden, case):
    import udpspeeder_amd as u
    k, n, ln, ng = case
    S = stride_for(ln)
    buf = np.zeros((ng, n, S), np.uint8)
    buf[:, :k, :ln] = group_data(DATA_SEED, 0, ng, k, ln)
    buf[:, k:] = 0xEE  # parity slots start as junk
    t = upload(buf, gpu)
    u.encode(t, k, n, ln)
    out = t.cpu().numpy()
    assert (out[:, k:, :ln] == golden.enc[f"parity_{k}_{n}_{ln}_{ng}"]).all()
    assert (out[:, :k] == buf[:, :k]).all()  # data untouched


@pytest.mark.parametrize("k,n,ln", [(20, 30, 1250), (20, 30, 1280), (5, 9, 300), (17, 27, 1100),
                                    (30, 40, 2000), (4, 20, 64), (64, 128, 96),
                                    (2, 255, 33), (1, 2, 5000)])
def test_encode_vs_oracle(gpu, oracle, k, n, ln):
    import udpspeeder_amd as u
    G = 37
    S = stride_for(ln) + 32  # stride larger than needed: padding must be ignored
    rng = np.random.default_rng(k * 1000 + n)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    t = upload(buf, gpu)
    u.encode(t, k, n, ln)
    oracle.encode_batch(k, n, buf.reshape(-1), n * S, S, ln, G)
    out = t.cpu().numpy()
    assert (out[:, :, :ln] == buf[:, :, :ln]).all()
    # bytes past the padding bound in every slot are never written
    pad = pad_end(ln, S)
    assert (out[:, :, pad:] == buf[:, :, pad:]).all()


def test_encode_c1_full_sha(gpu, golden):
    """C1: RS(20,10), 1250-B shards, 65536 groups; sha256 of data and parity
    equals the reference's (tests/golden/full_hashes.json)."""
    import torch
    import udpspeeder_amd as u
    F = golden.full["c1_encode"]
    k, n, ln, G = F["k"], F["n"], F["len"], F["groups"]
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, F["seed"])
    u.encode(t, k, n, ln)
    torch.cuda.synchronize()
    h_d = hashlib.sha256(); h_p = hashlib.sha256()
    for g0 in range(0, G, 8192):
        blk = t[g0:g0 + 8192, :, :ln].cpu().numpy()
        h_d.update(np.ascontiguousarray(blk[:, :k]).tobytes())
        h_p.update(np.ascontiguousarray(blk[:, k:]).tobytes())
    assert h_d.hexdigest() == F["data_sha256"]
    assert h_p.hexdigest() == F["parity_sha256"]


def _split_codes():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "udpspeeder_amd", "csrc"))
    import gen_bitslice as gb
    return [c for c in gb.default_codes() if gb.split_ok(*c)]


@pytest.mark.parametrize("k,n", _split_codes())
def test_encode_split_k_codes(gpu, oracle, k, n):
    """Every code with a split-k network (two waves per chunk, partial parities
    swapped over LDS): odd lengths, a ragged last chunk, against the oracle."""
    import udpspeeder_amd as u
    for G, ln in ((41, 1250), (7, 333), (1, 16)):
        S = stride_for(ln)
        rng = np.random.default_rng(k * 257 + n + ln)
        buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
        t = upload(buf, gpu)
        u.encode(t, k, n, ln)
        oracle.encode_batch(k, n, buf.reshape(-1), n * S, S, ln, G)
        out = t.cpu().numpy()
        assert (out[:, :, :ln] == buf[:, :, :ln]).all(), (G, ln)
        pad = pad_end(ln, S)
        assert (out[:, :, pad:] == buf[:, :, pad:]).all(), (G, ln)
    from udpspeeder_amd._lib import ENC_BITSLICE
    assert u.lib().rsmi_last_encoder() == ENC_BITSLICE


@pytest.mark.parametrize("bitslice", [True, False])
@pytest.mark.parametrize("k,n,ln", [(20, 30, 1250), (13, 21, 700), (1, 11, 64), (5, 15, 17)])
def test_encode_paths_agree(gpu, oracle, bitslice, k, n, ln):
    """The specialised bit-sliced and the generic kernels both match the oracle
    (these codes have a specialised kernel; bitslice=False forces generic)."""
    import udpspeeder_amd as u
    G = 333
    S = stride_for(ln)
    rng = np.random.default_rng(k + ln)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    t = upload(buf, gpu)
    prev = u.rs.set_bitslice(bitslice)
    try:
        u.encode(t, k, n, ln)
    finally:
        u.rs.set_bitslice(prev)
    oracle.encode_batch(k, n, buf.reshape(-1), n * S, S, ln, G)
    out = t.cpu().numpy()
    assert (out[:, :, :ln] == buf[:, :, :ln]).all()
    pad = pad_end(ln, S)
    assert (out[:, :, pad:] == buf[:, :, pad:]).all()


def test_encode_degenerate(gpu, oracle):
    import torch
    import udpspeeder_amd as u
    # k == n: nothing to do; len 0: nothing; zero groups
    t = torch.full((3, 4, 16), 7, dtype=torch.uint8, device=gpu)
    u.encode(t, 4, 4, 16)
    u.encode(t, 2, 4, 0)
    u.encode(t[:0], 2, 4, 16)
    assert (t.cpu().numpy() == 7).all()
    # RS(1,m) is replication
    buf = np.random.default_rng(3).integers(0, 256, (5, 4, 32), dtype=np.uint8)
    tt = upload(buf, gpu)
    u.encode(tt, 1, 4, 32)
    out = tt.cpu().numpy()
    assert (out[:, 1:] == out[:, :1]).all()


def test_encode_bad_args(gpu):
    import torch
    import udpspeeder_amd as u
    t = torch.zeros((2, 30, 1250), dtype=torch.uint8, device=gpu)  # stride not 16-aligned
    with pytest.raises(u.RsmiError):
        u.encode(t, 20, 30, 1250)
    t = torch.zeros((2, 30, 1280), dtype=torch.uint8, device=gpu)
    with pytest.raises(u.RsmiError):
        u.encode(t, 20, 19, 1250)
    with pytest.raises(u.RsmiError):
        u.encode(t, 20, 30, 1300)  # len > stride


# ---------------------------------------------------------------- decode
@pytest.mark.parametrize("name", _decode_cases())
def test_decode_small_golden(gpu, golden, name):
    import udpspeeder_amd as u
    D = golden.dec
    k, n, ln, ng, codeword = [int(x) for x in D[f"{name}__meta"]]
    present = D[f"{name}__present"]
    S = stride_for(ln)
    buf = np.zeros((ng, n, S), np.uint8)
    buf[:, :k, :ln] = group_data(DATA_SEED, 0, ng, k, ln)
    if codeword:
        u.encode(t0 := upload(buf, gpu), k, n, ln)
        buf = t0.cpu().numpy()
    else:
        buf[:, k:, :ln] = group_data(DATA_SEED ^ 0xFFFF, 0, ng, n - k, ln)
    assert sha(buf[:, :, :ln]) == D[f"{name}__input_sha"].tobytes().hex()
    buf[present == 0] = 0xA5  # erased slots hold junk that must never be read
    t = upload(buf, gpu)
    st = u.decode(t, upload(present, gpu), k, n, ln).cpu().numpy()
    out = t.cpu().numpy()
    assert (st == D[f"{name}__status"]).all()
    ok = st == 0
    assert sha(out[:, :k, :ln]) == D[f"{name}__data_out_sha"].tobytes().hex()
    rec = [out[g, j, :ln] for g in range(ng) if ok[g] for j in range(k) if not present[g, j]]
    rec = np.stack(rec) if rec else np.zeros((0, ln), np.uint8)
    assert (rec == D[f"{name}__recovered"]).all()
    assert (out[:, k:] == buf[:, k:]).all()  # parity slots untouched


@pytest.mark.parametrize("k,n,ln,ner", [(20, 30, 1250, 5), (20, 30, 1250, 10), (7, 13, 999, 6),
                                        (1, 4, 77, 3), (64, 128, 48, 64), (3, 6, 3, 3),
                                        (10, 16, 4096, 6), (2, 255, 20, 253)])
def test_decode_vs_oracle_random(gpu, oracle, k, n, ln, ner):
    import udpspeeder_amd as u
    G = 41
    S = stride_for(ln)
    rng = np.random.default_rng(k + n + ln)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)  # non-codeword: selection matters
    present = np.ones((G, n), np.uint8)
    for g in range(G):
        e = rng.integers(0, ner + 2)  # sometimes too many erasures -> -1
        present[g, rng.choice(n, min(e, n), replace=False)] = 0
    ref = buf.copy()
    st_ref = oracle.decode_batch(k, n, ref.reshape(-1), n * S, S, ln, G, present)
    t = upload(buf, gpu)
    st = u.decode(t, upload(present, gpu), k, n, ln).cpu().numpy()
    assert (st == st_ref).all()
    out = t.cpu().numpy()
    # data rows match the reference; parity slots are left untouched by the
    # batched contract (the reference overwrites the parity buffers it used)
    assert (out[:, :k, :ln] == ref[:, :k, :ln]).all()
    assert (out[:, k:] == buf[:, k:]).all()


@pytest.mark.parametrize("G", [4095, 50001, 65537, 131071])
def test_decode_grid_sizes(gpu, oracle, G):
    """Batch sizes that split unevenly over the fused decode's persistent grid
    (2,048 blocks at most: 1 to 16 groups per wave, some waves one group short).
    Round 2 dropped this test when the GPU test process crashed at exit with it
    in the suite; the cause was run-time compiles still inside hipRTC at exit
    (tests/test_bitslice_rtc.py::test_exit_during_compile_*), not this kernel."""
    import udpspeeder_amd as u
    k, n, ln = 20, 30, 48
    S = stride_for(ln)
    rng = np.random.default_rng(G)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    present = np.ones((G, n), np.uint8)
    er = np.argsort(rng.random((G, n)), axis=1)[:, :5]
    np.put_along_axis(present, er, 0, axis=1)
    ref = buf.copy()
    st_ref = oracle.decode_batch(k, n, ref.reshape(-1), n * S, S, ln, G, present)
    t = upload(buf, gpu)
    st = u.decode(t, upload(present, gpu), k, n, ln).cpu().numpy()
    assert (st == st_ref).all()
    out = t.cpu().numpy()
    assert (out[:, :k, :ln] == ref[:, :k, :ln]).all()
    # nothing outside the rebuilt rows' slots changed: parity rows and the
    # survivors are the input bytes
    assert (out[:, k:] == buf[:, k:]).all()


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("k,n,ln", [(20, 30, 1250), (20, 30, 3000), (7, 13, 100), (1, 2, 1280),
                                    (10, 20, 1281), (40, 50, 64)])
def test_decode_paths_agree(gpu, oracle, fused, k, n, ln):
    """Fused (one wave per group) and two-kernel decode both match the oracle,
    including lengths that need several 1280-B tiles and ragged tails."""
    import udpspeeder_amd as u
    G = 257
    S = stride_for(ln)
    rng = np.random.default_rng(k * n + ln)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    present = np.ones((G, n), np.uint8)
    for g in range(G):
        present[g, rng.choice(n, rng.integers(0, n - k + 2), replace=False)] = 0
    ref = buf.copy()
    st_ref = oracle.decode_batch(k, n, ref.reshape(-1), n * S, S, ln, G, present)
    t = upload(buf, gpu)
    prev = u.rs.set_fused_decode(fused)
    try:
        st = u.decode(t, upload(present, gpu), k, n, ln).cpu().numpy()
    finally:
        u.rs.set_fused_decode(prev)
    assert (st == st_ref).all()
    out = t.cpu().numpy()
    assert (out[:, :k, :ln] == ref[:, :k, :ln]).all()
    assert (out[:, k:] == buf[:, k:]).all()
    pad = pad_end(ln, S)
    assert (out[:, :, pad:] == buf[:, :, pad:]).all()


def test_decode_c2_full_noncodeword_sha(gpu, golden):
    """C2 at full size with random (non-codeword) parity: the recovered data
    rows hash to the reference's digest -- pins the survivor-selection rule
    over 65536 random 5-of-30 patterns."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    F = golden.full["c2_decode_noncodeword"]
    k, n, ln, G = F["k"], F["n"], F["len"], F["groups"]
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, DATA_SEED)
    u.fill_data(t[:, k:], n - k, ln, F["parity_seed"])
    pres = synth.erasure_present(F["erase_seed"], 0, G, n, F["erasures"])
    st = u.decode(t, upload(pres, gpu), k, n, ln)
    assert int((st != 0).sum().item()) == 0
    h = hashlib.sha256()
    for g0 in range(0, G, 8192):
        h.update(np.ascontiguousarray(t[g0:g0 + 8192, :k, :ln].cpu().numpy()).tobytes())
    assert h.hexdigest() == F["data_out_sha256"]


def test_roundtrip_full_c2(gpu):
    """encode -> erase 5 of 30 (poisoned) -> decode == original data, 65536 groups."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 1250, 65536
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, 1234)
    u.encode(t, k, n, ln)
    orig = t[:, :k, :ln].clone()
    pres = upload(synth.erasure_present(99, 0, G, n, 5), gpu)
    t.masked_fill_((pres == 0).unsqueeze(-1), 0x5A)
    st = u.decode(t, pres, k, n, ln)
    assert int((st != 0).sum().item()) == 0
    assert torch.equal(t[:, :k, :ln], orig)


# ---------------------------------------------------------------- ragged (C3)
def test_ragged_c3_full_sha(gpu, golden):
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    F = golden.full["c3_ragged_encode"]
    table = u.rs_from_str(F["fec"])
    ks, ms, ls = synth.ragged_mix(F["ragged_seed"], 0, F["groups"], [y for _, y in table],
                                  F["kmax"], F["len_min"], F["len_max"])
    groups, total = u.make_groups(ks, ks + ms, ls)
    base = torch.zeros(total, dtype=torch.uint8, device=gpu)
    dg = u.rs.groups_to_device(groups, gpu)
    u.rs.fill_ragged(base, dg, len(groups), DATA_SEED)
    u.encode_ragged(base, groups)
    host = base.cpu().numpy()
    h = hashlib.sha256()
    for i in range(len(groups)):
        d = groups[i]
        for j in range(d.k, d.n):
            o = d.offset + j * d.shard_stride
            h.update(host[o:o + d.len].tobytes())
    assert h.hexdigest() == F["parity_sha256"]


def test_ragged_vs_oracle_mixed(gpu, oracle):
    import torch
    import udpspeeder_amd as u
    rng = np.random.default_rng(5)
    G = 300
    ks = rng.integers(1, 40, G)
    ns = ks + rng.integers(0, 30, G)
    ls = rng.integers(0, 3000, G)
    groups, total = u.make_groups(ks, ns, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    base = upload(host, gpu)
    u.encode_ragged(base, groups)
    out = base.cpu().numpy()
    for i in range(G):
        d = groups[i]
        seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
        oracle.encode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1)
        got = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
        assert (got[:, :d.len] == seg.reshape(d.n, d.shard_stride)[:, :d.len]).all(), i


def test_ragged_bitslice_plan_vs_oracle(gpu, oracle):
    """Every group's code has a specialised network -> one bucketed bit-sliced
    launch; ragged lengths incl. 0, 1, 15, 16, 17 and > 1280; plan reuse."""
    import torch
    import udpspeeder_amd as u
    rng = np.random.default_rng(9)
    codes = [(x, x + 10) for x in range(1, 21)] + [(10, 16), (3, 8), (13, 21)]
    G = 2000
    pick = rng.integers(0, len(codes), G)
    ks = np.array([codes[i][0] for i in pick]); ns = np.array([codes[i][1] for i in pick])
    ls = rng.integers(0, 3000, G)
    ls[:6] = [0, 1, 15, 16, 17, 1280]
    groups, total = u.make_groups(ks, ns, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    base = upload(host, gpu)
    plan = u.rs.RaggedPlan(groups)
    assert plan.bitslice
    plan.encode(base)
    plan.encode(base)  # idempotent: parity depends only on data rows
    out = base.cpu().numpy()
    plan.close()
    for i in range(G):
        d = groups[i]
        seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
        oracle.encode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1)
        got = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
        exp = seg.reshape(d.n, d.shard_stride)
        assert (got[:, :d.len] == exp[:, :d.len]).all(), i
        pad = pad_end(d.len, d.shard_stride)
        assert (got[:, pad:] == host[d.offset:d.offset + d.n * d.shard_stride]
                .reshape(d.n, d.shard_stride)[:, pad:]).all(), i


def _ragged_noncodeword(gpu, ks, ms, ls, parity_seed):
    """Ragged batch on the GPU: data rows = DATA_SEED stream, parity rows =
    parity_seed stream (fill_ragged on descriptors that start at row k)."""
    import torch
    import udpspeeder_amd as u
    groups, total = u.make_groups(ks, ks + ms, ls)
    base = torch.zeros(total, dtype=torch.uint8, device=gpu)
    u.rs.fill_ragged(base, u.rs.groups_to_device(groups, gpu), len(groups), DATA_SEED)
    par, _ = u.make_groups(np.maximum(ms, 1), np.maximum(ms, 1), ls)
    for i in range(len(groups)):
        par[i].offset = groups[i].offset + groups[i].k * groups[i].shard_stride
        par[i].shard_stride = groups[i].shard_stride
    u.rs.fill_ragged(base, u.rs.groups_to_device(par, gpu), len(groups), parity_seed)
    return groups, base


def test_ragged_decode_c3_full_sha(gpu, golden):
    """C3 decode: the reference's full-size ragged non-codeword digest through
    one ragged plan (k_decode_ragged)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    F = golden.full["c3_ragged_decode"]
    table = u.rs_from_str(F["fec"])
    ks, ms, ls = synth.ragged_mix(F["ragged_seed"], 0, F["groups"], [y for _, y in table])
    groups, base = _ragged_noncodeword(gpu, ks, ms, ls, F["parity_seed"])
    flags = synth.ragged_erasures(F["erase_seed"], 0, ks + ms, ms, F["erasures"])
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    host = base.cpu().numpy()
    for i in range(len(groups)):  # erased slots hold junk: the decode must not read them
        d = groups[i]
        for j in np.nonzero(flags[i, :d.n] == 0)[0]:
            host[d.offset + j * d.shard_stride:d.offset + j * d.shard_stride + d.len] = 0x77
    base.copy_(torch.from_numpy(host))
    plan = u.rs.RaggedPlan(groups)
    st = plan.decode(base, bits)
    torch.cuda.synchronize()
    plan.close()
    assert int((st != 0).sum()) == 0
    out = base.cpu().numpy()
    h = hashlib.sha256()
    for i in range(len(groups)):
        d = groups[i]
        h.update(out[d.offset:d.offset + d.k * d.shard_stride].reshape(d.k, d.shard_stride)
                 [:, :d.len].tobytes())
    assert h.hexdigest() == F["data_out_sha256"]


def test_ragged_decode_vs_oracle_mixed(gpu, oracle):
    """Random codes (small and big: e > 10 and k > 64 go to the workgroup
    kernel), random lengths incl. 0/1/17/3000, random erasure counts incl.
    too few; every group against the C oracle, padding rule checked."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    rng = np.random.default_rng(21)
    G = 600
    ks = rng.integers(1, 40, G)
    ms = rng.integers(0, 30, G)
    ks[:40] = rng.integers(60, 200, 40)
    ms[:40] = rng.integers(1, 56, 40)
    ls = rng.integers(0, 3000, G)
    ls[40:46] = [0, 1, 17, 1280, 1281, 3000]
    groups, total = u.make_groups(ks, ks + ms, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    flags = np.zeros((G, 256), np.uint8)
    for i in range(G):
        n = int(ks[i] + ms[i])
        flags[i, :n] = 1
        ne = int(rng.integers(0, ms[i] + 2))  # sometimes one too many
        flags[i, rng.choice(n, min(ne, n), replace=False)] = 0
    base = upload(host, gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    st = u.rs.decode_ragged(base, groups, bits).cpu().numpy()
    out = base.cpu().numpy()
    for i in range(G):
        d = groups[i]
        n, k = d.n, d.k
        seg = host[d.offset:d.offset + n * d.shard_stride].copy()
        ost = oracle.decode_batch(k, n, seg, 0, d.shard_stride, d.len, 1, flags[i:i + 1, :n])
        assert st[i] == ost[0], (i, k, n, st[i], ost[0])
        got = out[d.offset:d.offset + n * d.shard_stride].reshape(n, d.shard_stride)
        exp = seg.reshape(n, d.shard_stride)
        org = host[d.offset:d.offset + n * d.shard_stride].reshape(n, d.shard_stride)
        if st[i] == 0:
            assert (got[:k, :d.len] == exp[:k, :d.len]).all(), (i, k, n, d.len)
        pad = pad_end(d.len, d.shard_stride)
        assert (got[:, pad:] == org[:, pad:]).all(), i
        assert (got[k:] == org[k:]).all(), i  # parity slots untouched


def test_ragged_plan_decode_many_codes_vs_oracle(gpu, oracle):
    """Plan decode (the width-class kernels, 8-dword group records read out of
    registers) over groups of ~200 different codes against the oracle: every
    code's parity rows sit at their own device address, so the records'
    64-bit pointers and offsets are rebuilt from many different low dwords
    (a sign-extended low dword with bit 31 set faulted the GPU once)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    rng = np.random.default_rng(77)
    codes = sorted({(int(k), int(k + m)) for k, m in zip(rng.integers(1, 61, 400), rng.integers(1, 21, 400))})
    G = 3 * len(codes)
    pick = rng.integers(0, len(codes), G)
    ks = np.array([codes[i][0] for i in pick]); ns = np.array([codes[i][1] for i in pick])
    ls = rng.integers(1, 1300, G)
    groups, total = u.make_groups(ks, ns, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    flags = np.zeros((G, 256), np.uint8)
    for i in range(G):
        n, m = int(ns[i]), int(ns[i] - ks[i])
        flags[i, :n] = 1
        # up to 10 erasures, so e > 5 groups (and k > 32 ones) are deferred
        # to the workgroup kernel, whose launch the plan gates on a mark
        flags[i, rng.choice(n, min(int(rng.integers(1, 11)), m), replace=False)] = 0
    plan = u.rs.RaggedPlan(groups, wait_codes=False)
    base = upload(host, gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    st = plan.decode(base, bits).cpu().numpy()
    # a second call that defers nothing (all present), then the first again
    allp = torch.from_numpy(synth.present_bits((np.arange(256)[None, :] < ns[:, None]).astype(np.uint8))
                            .view(np.int32)).to(gpu)
    assert (plan.decode(base, allp).cpu().numpy() == 0).all()
    base.copy_(upload(host, gpu))
    st2 = plan.decode(base, bits).cpu().numpy()
    assert (st2 == st).all()
    plan.close()
    out = base.cpu().numpy()
    for i in range(G):
        d = groups[i]
        n, k = d.n, d.k
        seg = host[d.offset:d.offset + n * d.shard_stride].copy()
        ost = oracle.decode_batch(k, n, seg, 0, d.shard_stride, d.len, 1, flags[i:i + 1, :n])
        assert st[i] == ost[0], (i, k, n)
        got = out[d.offset:d.offset + n * d.shard_stride].reshape(n, d.shard_stride)
        assert (got[:k, :d.len] == seg.reshape(n, d.shard_stride)[:k, :d.len]).all(), (i, k, n)


def test_ragged_decode_offsets_bit31(gpu, oracle):
    """Round-3 fault, pinned on purpose: the class kernels rebuild a group's
    64-bit offset from two record dwords read with v_readlane, and a low dword
    with bit 31 set once sign-extended into the high half (commit 83459b6).
    Here every group of the batch sits past 2 GiB inside one tensor (offsets
    0x8000_0000 + ..., low dword bit 31 set), and the batch decodes through a
    plan (k_decode_ragged_cls, plus the workgroup kernel for e > 5) and
    through the device-descriptor form (k_decode_ragged), both against the
    oracle.  Before the fix this faulted the GPU; now it must be bit-exact."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    rng = np.random.default_rng(31)
    G = 400
    ks = rng.integers(1, 21, G)
    ms = rng.integers(1, 11, G)
    ls = rng.integers(1, 1300, G)  # every tile-width class
    groups, total = u.make_groups(ks, ks + ms, ls)
    shift = 0x80000000 + 4096
    for i in range(G):
        groups[i].offset += shift
        assert (groups[i].offset & 0xFFFFFFFF) >> 31 == 1
    host = rng.integers(0, 256, total, dtype=np.uint8)
    flags = np.zeros((G, 256), np.uint8)
    for i in range(G):
        n = int(ks[i] + ms[i])
        flags[i, :n] = 1
        ne = min(int(rng.integers(1, 8)), int(ms[i]))  # some e > 5: deferred groups too
        flags[i, rng.choice(n, ne, replace=False)] = 0
    for c in set(zip(ks.tolist(), (ks + ms).tolist())):
        u.prepare_code(*c)
    base = torch.zeros(shift + total, dtype=torch.uint8, device=gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    exp, ost = host.copy(), np.zeros(G, np.int32)
    for i in range(G):
        d = groups[i]
        o = d.offset - shift
        seg = exp[o:o + d.n * d.shard_stride]
        ost[i] = oracle.decode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1,
                                     flags[i:i + 1, :d.n])[0]
        exp[o:o + d.n * d.shard_stride] = seg
    plan = u.rs.RaggedPlan(groups, wait_codes=False)
    dgroups = u.rs.groups_to_device(groups, gpu)
    for form in ("plan", "dev"):
        base[shift:].copy_(torch.from_numpy(host).to(gpu))
        if form == "plan":
            st = plan.decode(base, bits)
        else:
            st = u.rs.decode_ragged_dev(base, dgroups, G, bits, kmax=20)
        st = st.cpu().numpy()
        out = base[shift:].cpu().numpy()
        assert (base[:shift].count_nonzero().item()) == 0, form  # nothing written below the groups
        assert (st == ost).all(), form
        for i in range(G):
            d = groups[i]
            o = d.offset - shift
            got = out[o:o + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
            ref = exp[o:o + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
            assert (got[:d.k, :d.len] == ref[:d.k, :d.len]).all(), (form, i)
    plan.close()


@pytest.mark.parametrize("cap", [1, 3])
def test_ragged_plan_decode_record_cap(gpu, oracle, cap):
    """A plan's decode workgroups stage their group records in LDS, capped to
    the class kernels' LDS budget (ragged.cpp); past the cap the plan deals
    the groups to more workgroups than one resident round.  Forcing a cap of
    1 or 3 records (RSMI_OPT_CLS_REC_CAP) makes a 6,000-group plan run every
    width class over many rounds of workgroups: bit-exact with the oracle."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    from udpspeeder_amd._lib import RSMI_OPT_CLS_REC_CAP
    rng = np.random.default_rng(50 + cap)
    G = 6000
    ks = rng.integers(1, 21, G)
    ms = rng.integers(1, 11, G)
    ls = rng.integers(1, 1300, G)
    groups, total = u.make_groups(ks, ks + ms, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    flags = np.zeros((G, 256), np.uint8)
    for i in range(G):
        n = int(ks[i] + ms[i])
        flags[i, :n] = 1
        flags[i, rng.choice(n, min(5, int(ms[i])), replace=False)] = 0
    L = u.lib()
    prev = L.rsmi_option(RSMI_OPT_CLS_REC_CAP, cap)
    try:
        plan = u.rs.RaggedPlan(groups, wait_codes=False)
    finally:
        L.rsmi_option(RSMI_OPT_CLS_REC_CAP, prev)
    base = upload(host, gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    st = plan.decode(base, bits).cpu().numpy()
    plan.close()
    out = base.cpu().numpy()
    for i in range(G):
        d = groups[i]
        n, k = d.n, d.k
        seg = host[d.offset:d.offset + n * d.shard_stride].copy()
        ost = oracle.decode_batch(k, n, seg, 0, d.shard_stride, d.len, 1, flags[i:i + 1, :n])
        assert st[i] == ost[0], (i, k, n)
        got = out[d.offset:d.offset + n * d.shard_stride].reshape(n, d.shard_stride)
        assert (got[:k, :d.len] == seg.reshape(n, d.shard_stride)[:k, :d.len]).all(), (i, k, n)


def test_ragged_plan_decode_graph_capture(gpu, oracle):
    """A ragged plan decode forks its width classes over extra streams and joins
    them back (event fork/join): it captures into a graph, and every replay
    matches the oracle on the batch's current contents."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    rng = np.random.default_rng(33)
    G = 700
    ks = rng.integers(1, 21, G)
    ms = rng.integers(1, 11, G)
    ls = rng.integers(1, 1300, G)  # all four tile widths
    groups, total = u.make_groups(ks, ks + ms, ls)
    flags = np.zeros((G, 256), np.uint8)
    for i in range(G):
        n = int(ks[i] + ms[i])
        flags[i, :n] = 1
        flags[i, rng.choice(n, min(5, int(ms[i])), replace=False)] = 0
    plan = u.rs.RaggedPlan(groups, wait_codes=False)  # decode needs no encode networks
    base = torch.zeros(total, dtype=torch.uint8, device=gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    st = torch.empty(G, dtype=torch.int32, device=gpu)
    plan.decode(base, bits, status=st)  # warm-up outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        plan.decode(base, bits, status=st)
    for seed in (4, 5):
        host = np.random.default_rng(seed).integers(0, 256, total, dtype=np.uint8)
        base.copy_(torch.from_numpy(host).to(gpu))
        st.fill_(7)
        g.replay()
        torch.cuda.synchronize()
        out = base.cpu().numpy()
        sts = st.cpu().numpy()
        for i in range(0, G, 7):
            d = groups[i]
            n, k = d.n, d.k
            seg = host[d.offset:d.offset + n * d.shard_stride].copy()
            ost = oracle.decode_batch(k, n, seg, 0, d.shard_stride, d.len, 1, flags[i:i + 1, :n])
            assert sts[i] == ost[0], (seed, i)
            got = out[d.offset:d.offset + n * d.shard_stride].reshape(n, d.shard_stride)
            assert (got[:k, :d.len] == seg.reshape(n, d.shard_stride)[:k, :d.len]).all(), (seed, i)


def test_ragged_decode_dev_unresident_code(gpu, oracle):
    """The device-descriptor form: resident codes decode, a code that was
    never made resident reports RSMI_DEC_UNSUPPORTED and is left alone."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    from udpspeeder_amd._lib import RSMI_DEC_UNSUPPORTED
    ks = np.array([20, 13, 251]); ms = np.array([10, 7, 3]); ls = np.array([1250, 700, 100])
    u.prepare_code(20, 30)
    u.prepare_code(13, 20)
    groups, total = u.make_groups(ks, ks + ms, ls)
    rng = np.random.default_rng(2)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    flags = np.zeros((3, 256), np.uint8)
    for i in range(3):
        flags[i, :ks[i] + ms[i]] = 1
        flags[i, [0, 2]] = 0
    base = upload(host, gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    st = u.rs.decode_ragged_dev(base, u.rs.groups_to_device(groups, gpu), 3, bits, kmax=20)
    st = st.cpu().numpy()
    out = base.cpu().numpy()
    assert st.tolist() == [0, 0, RSMI_DEC_UNSUPPORTED]
    d = groups[2]
    assert (out[d.offset:d.offset + d.n * d.shard_stride] ==
            host[d.offset:d.offset + d.n * d.shard_stride]).all()
    for i in range(2):
        d = groups[i]
        seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
        oracle.decode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1, flags[i:i + 1, :d.n])
        got = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
        assert (got[:d.k, :d.len] == seg.reshape(d.n, d.shard_stride)[:d.k, :d.len]).all()


# ---------------------------------------------------------------- drop-in shim
def test_compat_kat_misc_unit_test(gpu, golden):
    """misc.cpp:335-361 through the reference-mangled rs_encode2/rs_decode2."""
    import udpspeeder_amd as u
    kat = golden.kat
    arr = [bytearray(b"aaa" + bytes(97)), bytearray(b"bbb" + bytes(97)),
           bytearray(b"ccc" + bytes(97)), bytearray(b"ddd" + bytes(97)),
           bytearray(b"eee" + bytes(97)), bytearray(b"fff" + bytes(97))]
    data = list(arr)
    u.rs_encode2(3, 6, data, 3)
    assert [bytes(data[i][:3]).hex() for i in range(3, 6)] == kat["parity"]
    data[0] = None
    rc = u.rs_decode2(3, 6, data, 3)
    assert rc == kat["decode_rc"] == 0
    slots = [next((i for i, a in enumerate(arr) if a is d), -1) if d is not None else -1
             for d in data]
    assert slots == kat["decode_out_slots"]
    assert [bytes(d[:3]).hex() if d is not None else None for d in data] == kat["decode_out_bytes"]


@pytest.mark.parametrize("name", _decode_cases())
def test_compat_pointer_permutation(gpu, golden, name):
    import udpspeeder_amd as u
    D = golden.dec
    k, n, ln, ng, codeword = [int(x) for x in D[f"{name}__meta"]]
    if codeword:
        pytest.skip("pointer cases use non-codeword inputs")
    present = D[f"{name}__present"][0]
    data = group_data(DATA_SEED, 0, 1, k, ln)[0]
    par = group_data(DATA_SEED ^ 0xFFFF, 0, 1, n - k, ln)[0]
    rows = [bytearray(r.tobytes()) for r in np.concatenate([data, par])] if ln else \
        [bytearray(1) for _ in range(n)]
    arr = [bytearray(r) for r in rows]
    ptrs = [arr[j] if present[j] else None for j in range(n)]
    rc = u.rs_decode2(k, n, ptrs, ln)
    assert rc == int(D[f"{name}__ptr_rc"][0])
    slots = [next((i for i, a in enumerate(arr) if a is p), -1) if p is not None else -1
             for p in ptrs]
    assert slots == D[f"{name}__ptr_out"].tolist()
    after = np.stack([np.frombuffer(bytes(a[:ln]), np.uint8) for a in arr]) if ln else \
        np.zeros((n, 0), np.uint8)
    assert sha(after) == D[f"{name}__ptr_bufs_sha"].tobytes().hex()


@pytest.mark.parametrize("one_group", [True, False])
@pytest.mark.parametrize("k,n,ln", [(20, 30, 1250), (3, 6, 3), (1, 2, 1), (40, 60, 700),
                                    (10, 16, 5000), (128, 255, 64), (7, 13, 100), (20, 30, 17),
                                    (60, 70, 300), (20, 52, 200)])
def test_dropin_one_group_vs_oracle(gpu, oracle, one_group, k, n, ln):
    """rs_encode2 / rs_decode2 of one group on non-codeword inputs, through
    the one-kernel latency path (RSMI_OPT_ONE_GROUP, oneshot.hip: pinned
    staging read over PCIe, completion flag) and through the staged copy path:
    both bit-exact with the oracle.  Covers survivors beyond one register
    chunk (k = 40), shards longer than 4 KiB (several column blocks), e > 8
    (several row blocks), a code outside the kernel's LDS budget (k = 128,
    n = 255: it falls back), and the whole-workgroup LDS elimination of
    oneshot.hip: (60, 70) with e = 5 and 9 has e + k > 64 columns, (20, 52)
    with e = 13 and 20 has more than 10 rows."""
    import udpspeeder_amd as u
    L = u.lib()
    prev = L.rsmi_option(3, int(one_group))
    try:
        rng = np.random.default_rng(k * 31 + n + ln)
        es = [1, 5, 9] + ([13, 20] if min(k, n - k) > 10 else [])
        for trial, e_want in enumerate(es):
            rows = rng.integers(0, 256, (n, ln), dtype=np.uint8)
            # encode
            data = [bytearray(rows[j].tobytes()) for j in range(n)]
            u.rs_encode2(k, n, data, ln)
            ref = np.zeros((n, ln), np.uint8)
            ref[:k] = rows[:k]
            oracle.encode_batch(k, n, ref.reshape(-1), 0, ln, ln, 1)
            for j in range(n):
                assert bytes(data[j]) == ref[j].tobytes(), ("encode", trial, j)
            # decode a non-codeword: up to min(k, m) erasures, data first
            m = n - k
            e = min(k, m, e_want)
            er = [int(x) for x in rng.choice(k, e, replace=False)]
            if m > e:  # and one parity shard, so the survivors skip it
                er.append(k + int(rng.integers(0, m)))
            present = np.ones(n, np.uint8)
            present[er] = 0
            buf = np.ascontiguousarray(rows.copy())
            st_ref = oracle.decode_batch(k, n, buf.reshape(-1), 0, ln, ln, 1, present[None, :])
            arr = [bytearray(rows[j].tobytes()) for j in range(n)]
            ptrs = [arr[j] if present[j] else None for j in range(n)]
            rc = u.rs_decode2(k, n, ptrs, ln)
            assert rc == int(st_ref[0])
            for j in range(k):
                assert bytes(ptrs[j]) == buf[j].tobytes(), ("decode", trial, j)
    finally:
        L.rsmi_option(3, prev)


def test_compat_lower_api(gpu, oracle):
    import udpspeeder_amd as u
    k, n, ln = 5, 9, 40
    rng = np.random.default_rng(11)
    rows = [bytearray(rng.integers(0, 256, ln, dtype=np.uint8).tobytes()) for _ in range(n)]
    code = u.fec_new(k, n)
    assert code and u.get_k(code) == k and u.get_n(code) == n
    assert u.fec_new(3, 2) is None and u.fec_new(257, 300) is None
    ref = np.zeros((n, ln), np.uint8)
    for j in range(k):
        ref[j] = np.frombuffer(bytes(rows[j]), np.uint8)
    oracle.encode_batch(k, n, ref.reshape(-1), 0, ln, ln, 1)
    for idx in range(n):
        dst = bytearray(ln)
        u.fec_encode(code, rows[:k], dst, idx, ln)
        assert bytes(dst) == ref[idx].tobytes(), idx
    enc = [bytearray(ref[j].tobytes()) for j in range(n)]
    u.rs_encode(code, [bytearray(ref[j].tobytes()) if j < k else enc[j] for j in range(n)], ln)
    # fec_decode with packets 1,2,5,7,8 (shuffled) recovers data rows 0,3,4
    pkt = [bytearray(ref[i].tobytes()) for i in (7, 1, 2, 8, 5)]
    index = [7, 1, 2, 8, 5]
    rc = u.fec_decode(code, pkt, index, ln)
    assert rc == 0
    for row in range(k):
        assert bytes(pkt[row]) == ref[row].tobytes()
    assert u.fec_decode(code, [bytearray(ln) for _ in range(5)], [1, 1, 2, 3, 4], ln) == 1
    u.fec_free(code)
    assert u.get_code(20, 30) == u.get_code(20, 30)


def test_encode_pinned_pipeline(gpu, oracle):
    import torch
    import udpspeeder_amd as u
    k, n, ln, G, S = 20, 30, 1250, 10000, 1280
    data = torch.from_numpy(group_data(DATA_SEED, 0, G, k, ln)).contiguous()
    d = torch.zeros((G, k, S), dtype=torch.uint8).pin_memory()
    d[:, :, :ln] = data
    par = torch.zeros((G, n - k, S), dtype=torch.uint8).pin_memory()
    u.rs.encode_pinned(d, par, k, n, ln, chunk_groups=1536)
    ref = np.zeros((G, n, S), np.uint8)
    ref[:, :k] = d.numpy()
    oracle.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G)
    assert (par.numpy()[:, :, :ln] == ref[:, k:, :ln]).all()


def test_decode_pinned_pipeline(gpu, oracle):
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G, S = 20, 30, 1250, 9000, 1280
    h = torch.zeros((G, n, S), dtype=torch.uint8).pin_memory()
    h[:, :k, :ln] = torch.from_numpy(group_data(DATA_SEED, 0, G, k, ln))
    t = h.cuda()
    u.encode(t, k, n, ln)
    h.copy_(t.cpu())
    orig = h[:, :k, :ln].clone()
    pres = synth.erasure_present(21, 0, G, n, 6)
    h[torch.from_numpy(pres == 0)] = 0xA5
    before = h.clone()
    st = u.rs.decode_pinned(h, pres, k, n, ln, chunk_groups=1000)
    assert u.lib().rsmi_last_decode_pinned_path() == 1  # zero-copy: pinned torch memory
    assert (st == 0).all()
    assert torch.equal(h[:, :k, :ln], orig)
    # only the rebuilt data rows were written: every other slot is as it was
    # (erased parity slots still hold the 0xA5 junk)
    rebuilt = torch.from_numpy(pres == 0)
    rebuilt[:, k:] = False
    assert torch.equal(h[~rebuilt], before[~rebuilt])


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("k,n,ln,S,off", [(20, 30, 1250, 1280, 0), (10, 16, 1283, 1296, 7),
                                          (7, 13, 100, 112, 3), (20, 30, 1250, 1280, 5)])
def test_decode_pinned_noncodeword(gpu, oracle, pinned, k, n, ln, S, off):
    """rsmi_decode_pinned on non-codewords (random parity, so the bytes pin
    which survivors are used, lib/rs.cpp:24-39) against the oracle: pinned
    torch memory (zero-copy path, also from an interior offset of the
    allocation) and pageable numpy memory (staged path)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    G = 1500
    rng = np.random.default_rng(k * 1000 + S + off)
    raw = rng.integers(0, 256, ((G + off) * n * S,), dtype=np.uint8)
    pres = synth.erasure_present(77 + k, 0, G, n, min(n - k, 6))
    ref = raw[off * n * S:].copy()
    st_ref = oracle.decode_batch(k, n, ref, n * S, S, ln, G, pres)
    if pinned:
        big = torch.from_numpy(raw).pin_memory()
        h = big[off * n * S:].view(G, n, S)  # an interior pointer of the pinned block
        st = u.rs.decode_pinned(h, pres, k, n, ln, chunk_groups=512)
        out = h.numpy().reshape(-1)
        want = 1
    else:
        h = raw[off * n * S:].reshape(G, n, S)
        st = u.rs.decode_pinned(h, pres, k, n, ln, chunk_groups=512)
        out = h.reshape(-1)
        want = 2
    assert u.lib().rsmi_last_decode_pinned_path() == want
    assert (st == st_ref).all()
    o = out.reshape(G, n, S)
    r = ref.reshape(G, n, S)
    assert (o[:, :k, :ln] == r[:, :k, :ln]).all()


def test_host_batched_api(gpu, oracle):
    import udpspeeder_amd as u
    k, n, ln, G = 20, 30, 1250, 64
    buf = np.zeros((G, n, 1300), np.uint8)
    buf[:, :k, :ln] = group_data(DATA_SEED, 0, G, k, ln)
    ref = buf.copy()
    u.encode_host(buf.reshape(-1), k, n, ln, n * 1300, 1300, G)
    oracle.encode_batch(k, n, ref.reshape(-1), n * 1300, 1300, ln, G)
    assert (buf == ref).all()
    from udpspeeder_amd import synth
    pres = synth.erasure_present(3, 0, G, n, 7)
    cor = buf.copy()
    cor[pres == 0] = 0
    st = u.decode_host(cor.reshape(-1), pres, k, n, ln, n * 1300, 1300, G)
    assert (st == 0).all()
    assert (cor[:, :k, :ln] == ref[:, :k, :ln]).all()


def test_hipgraph_capture_replay(gpu, oracle):
    """encode + fused decode are graph-capturable after prepare/reserve, and a
    replay recomputes from the current contents of the input buffers."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 1250, 512
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    pres = torch.from_numpy(synth.erasure_present(3, 0, G, n, 5)).to(gpu)
    st = torch.empty(G, dtype=torch.int32, device=gpu)
    u.fill_data(t, k, ln, 1)
    u.reserve(k, n, G)
    u.encode(t, k, n, ln)
    u.decode(t, pres, k, n, ln, status=st)  # warm-up outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        u.encode(t, k, n, ln)
        u.decode(t, pres, k, n, ln, status=st)
    for seed in (2, 3):
        u.fill_data(t, k, ln, seed)          # new data, same layout
        t[:, k:] = 0
        g.replay()
        torch.cuda.synchronize()
        host = t.cpu().numpy()
        ref = host.copy()
        ref[:, k:] = 0
        oracle.encode_batch(k, n, ref.reshape(-1), n * 1280, 1280, ln, G)
        assert (host[:, :, :ln] == ref[:, :, :ln]).all()
        assert int((st != 0).sum()) == 0


def test_concurrent_streams(gpu, oracle):
    """Two streams encoding/decoding different batches concurrently (no
    cross-stream ordering in librsmi): data rows and surviving parity rows."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 1250, 2048
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ts = [torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu) for _ in range(2)]
    for i, t in enumerate(ts):
        u.fill_data(t, k, ln, 100 + i)
    torch.cuda.synchronize()
    ref = [t.cpu().numpy() for t in ts]
    pres = [torch.from_numpy(synth.erasure_present(7 + i, 0, G, n, 5)).to(gpu) for i in range(2)]
    for _ in range(3):
        for t, s, p in zip(ts, (s1, s2), pres):
            with torch.cuda.stream(s):
                u.encode(t, k, n, ln)
                t.masked_fill_((p == 0).unsqueeze(-1), 0x77)
                u.decode(t, p, k, n, ln)
    torch.cuda.synchronize()
    for t, r, p in zip(ts, ref, pres):
        oracle.encode_batch(k, n, r.reshape(-1), n * 1280, 1280, ln, G)
        out = t.cpu().numpy()
        assert (out[:, :k, :ln] == r[:, :k, :ln]).all()
        keep = p.cpu().numpy()[:, k:] != 0
        assert (out[:, k:, :ln][keep] == r[:, k:, :ln][keep]).all()


def test_concurrent_streams_stress(gpu, oracle):
    """The two-stream encode -> erase -> decode scenario repeated from fresh
    inputs, checked on the GPU after every round.  With the parity stores'
    shard offset in soffset (round 1, BS_ST_SGPR=1) this found wrong first
    dwords in parity rows 20-21 in ~1 of 400 rounds."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G, reps = 20, 30, 1250, 2048, 1500
    init, want, pres = [], [], []
    for i in range(2):
        t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
        u.fill_data(t, k, ln, 200 + i)
        init.append(t)
        r = t.cpu().numpy()
        oracle.encode_batch(k, n, r.reshape(-1), n * 1280, 1280, ln, G)
        p = torch.from_numpy(synth.erasure_present(17 + i, 0, G, n, 5)).to(gpu)
        pres.append(p)
        w = torch.from_numpy(r).to(gpu)
        w.masked_fill_((p == 0).unsqueeze(-1), 0x77)   # erased parity rows stay 0x77
        w[:, :k] = torch.from_numpy(r[:, :k]).to(gpu)   # data rows all rebuilt
        want.append(w[:, :, :ln].contiguous())
    masks = [(p == 0).unsqueeze(-1) for p in pres]
    ts = [t.clone() for t in init]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    bad = torch.zeros(2, dtype=torch.int64, device=gpu)
    for _ in range(reps):
        for t, i0 in zip(ts, init):
            t.copy_(i0)
        torch.cuda.synchronize()
        for t, s, p, m in zip(ts, (s1, s2), pres, masks):
            with torch.cuda.stream(s):
                u.encode(t, k, n, ln)
                t.masked_fill_(m, 0x77)
                u.decode(t, p, k, n, ln)
        torch.cuda.synchronize()
        for i in range(2):
            bad[i] += (ts[i][:, :, :ln] != want[i]).sum()
    assert bad.tolist() == [0, 0]


def test_concurrent_ragged_and_decode(gpu, oracle):
    """A bucketed bit-sliced ragged encode on one stream beside uniform fused
    decodes on another (every launch path runs concurrently)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    rng = np.random.default_rng(31)
    codes = [(x, x + 10) for x in range(1, 21)]
    Gr = 3000
    pick = rng.integers(0, len(codes), Gr)
    ks = np.array([codes[i][0] for i in pick]); ns = np.array([codes[i][1] for i in pick])
    ls = rng.integers(64, 1251, Gr)
    groups, total = u.make_groups(ks, ns, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    base = upload(host, gpu)
    plan = u.rs.RaggedPlan(groups)
    k, n, ln, G = 20, 30, 1250, 4096
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, 77)
    u.encode(t, k, n, ln)
    torch.cuda.synchronize()
    clean = t.clone()
    p = torch.from_numpy(synth.erasure_present(5, 0, G, n, 8)).to(gpu)
    m = (p == 0).unsqueeze(-1)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(20):
        with torch.cuda.stream(s1):
            plan.encode(base)
        with torch.cuda.stream(s2):
            t.masked_fill_(m, 0x5A)
            u.decode(t, p, k, n, ln)
    torch.cuda.synchronize()
    plan.close()
    assert torch.equal(t[:, :k, :ln], clean[:, :k, :ln])
    out = base.cpu().numpy()
    for i in range(0, Gr, 7):
        d = groups[i]
        seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
        oracle.encode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1)
        got = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
        assert (got[:, :d.len] == seg.reshape(d.n, d.shard_stride)[:, :d.len]).all(), i


def test_decode_wrappers_reject_bad_status_and_masks(gpu):
    """The kernels write status[g] for every g < G and read 8 mask words per
    group: the Python wrappers refuse a short / wrong-dtype status tensor and
    a misshaped present_bits before anything is launched."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 64, 8
    t = torch.zeros((G, n, 64), dtype=torch.uint8, device=gpu)
    pres = torch.ones((G, n), dtype=torch.uint8, device=gpu)
    for bad in (torch.zeros(G - 1, dtype=torch.int32, device=gpu),
                torch.zeros(G, dtype=torch.int64, device=gpu)):
        with pytest.raises((ValueError, TypeError)):
            u.decode(t, pres, k, n, ln, status=bad)
    groups, total = u.make_groups([3] * G, [5] * G, [40] * G)
    base = torch.zeros(total, dtype=torch.uint8, device=gpu)
    flags = np.ones((G, 5), np.uint8)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    u.prepare_code(3, 5)
    with pytest.raises(ValueError):
        u.rs.decode_ragged(base, groups, bits[:G - 1])
    with pytest.raises(ValueError):
        u.rs.decode_ragged(base, groups, bits, status=torch.zeros(G - 1, dtype=torch.int32, device=gpu))
    dg = u.rs.groups_to_device(groups, gpu)
    with pytest.raises(ValueError):
        u.rs.decode_ragged_dev(base, dg[:24 * (G - 1)], G, bits)
    with pytest.raises(ValueError):
        u.rs.decode_ragged_dev(base, dg, G, bits, status=torch.zeros(2, dtype=torch.int32, device=gpu))
    st = u.rs.decode_ragged_dev(base, dg, G, bits, kmax=3)
    assert (st.cpu().numpy() == 0).all()
