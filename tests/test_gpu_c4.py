"""GPU: BASELINE configs[4] (C4) as far as one GPU covers it.

C4 is RS(20,10) encode + decode of 1250-B shards over 2^20 groups split across
8 GPUs.  FEC groups are independent (connection.h:244-245), so a
rank's work is exactly its contiguous slice shard.strong_range(r, 8, 2^20),
with the PRNG streams keyed by the GLOBAL group id.  These tests run two
ranks' slices (0/8, 3/8 at g0 = 393,216, 5/8 and 7/8 at g0 = 917,504) through the same
calls bench.py's ranks make, and check the bytes against sha256 digests the
real reference (lib/rs.cpp + lib/fec.cpp, oracle/_ref) produced for exactly
those slices (tests/golden/full_hashes.json "c4_rank_slices", made by
`python -m oracle.gen_golden --c4`).  A third test runs all 2^20 groups on
this one GPU: encode, poison the erased slots, decode, compare every data
byte with the original."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STRIDE = 1280


@pytest.mark.parametrize("rank", [0, 3, 5, 7])
def test_c4_rank_slice_encode_decode(gpu, golden, rank):
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import shard, synth
    F = golden.full["c4_rank_slices"]
    k, n, ln = F["k"], F["n"], F["len"]
    R = F["ranks"][str(rank)]
    g0, g1 = shard.strong_range(rank, F["world"], F["groups"])
    assert (g0, g1) == (R["g0"], R["g1"])
    G = g1 - g0
    t = torch.empty((G, n, STRIDE), dtype=torch.uint8, device=gpu)
    # encode: the rank's slice of the C4 data stream
    u.fill_data(t, k, ln, F["seed"], g0=g0)
    u.encode(t, k, n, ln)
    h = hashlib.sha256()
    for c in range(0, G, 16384):
        h.update(np.ascontiguousarray(t[c:c + 16384, k:, :ln].cpu().numpy()).tobytes())
    assert h.hexdigest() == R["parity_sha256"]
    # decode: non-codeword slice (random parity) pins which survivors are used
    u.fill_data(t, k, ln, F["seed"], g0=g0)
    u.fill_data(t[:, k:], n - k, ln, F["parity_seed"], g0=g0)
    pres = torch.from_numpy(synth.erasure_present(F["erase_seed"], g0, G, n, F["erasures"])).to(gpu)
    t.masked_fill_((pres == 0).unsqueeze(-1), 0xA5)  # erased slots hold junk
    st = u.decode(t, pres, k, n, ln)
    assert int((st != 0).sum().item()) == 0
    h = hashlib.sha256()
    for c in range(0, G, 16384):
        h.update(np.ascontiguousarray(t[c:c + 16384, :k, :ln].cpu().numpy()).tobytes())
    assert h.hexdigest() == R["data_out_sha256"]


def test_c4_all_groups_one_gpu_roundtrip(gpu, golden):
    """All 2^20 C4 groups resident on one GPU (40 GB of slots): encode, then
    lose 5 random shards per group (slots poisoned), decode, and every data
    byte equals the original; the parity of the rank-3 slice inside the big
    batch equals the reference's digest too (a slice at g0 = 393,216 of one
    launch, not its own launch)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 1250, 1 << 20
    t = torch.empty((G, n, STRIDE), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, synth.DATA_SEED)
    u.encode(t, k, n, ln)
    R = golden.full["c4_rank_slices"]["ranks"]["3"]
    h = hashlib.sha256()
    for c in range(R["g0"], R["g1"], 16384):
        h.update(np.ascontiguousarray(t[c:c + 16384, k:, :ln].cpu().numpy()).tobytes())
    assert h.hexdigest() == R["parity_sha256"]
    orig = t[:, :k, :ln].clone()
    pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, 0, G, n, 5)).to(gpu)
    t.masked_fill_((pres == 0).unsqueeze(-1), 0x3C)
    st = u.decode(t, pres, k, n, ln)
    assert int((st != 0).sum().item()) == 0
    assert torch.equal(t[:, :k, :ln], orig)
    del orig
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world,rank", [(1, 0), (4, 2), (8, 5)])
def test_bench_verify_slice(gpu, world, rank):
    """bench.py's after-the-timed-region check (verify_slice): a rank's C4
    slice, encoded and decoded through the bench's own calls, matches the
    reference's per-group-checksum digests for its range (N = 1's 65,536
    groups, rank 2 of 4, rank 5 of 8); a corrupted parity byte is caught."""
    import torch
    import bench
    import udpspeeder_amd as u
    from udpspeeder_amd import shard, synth
    k, n, ln = 20, 30, 1250
    g0, g1 = (0, 65536) if world == 1 else shard.strong_range(rank, world, 1 << 20)
    G = g1 - g0
    t = torch.empty((G, n, STRIDE), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, synth.DATA_SEED, g0=g0)
    pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, g0, G, n, 5)).to(gpu)
    u.encode(t, k, n, ln)
    u.decode(t, pres, k, n, ln)
    r = bench.verify_slice(u, synth, torch, t, pres, g0, G)
    assert r["ok"] is True, r
    u.fill_data(t, k, ln, synth.DATA_SEED, g0=g0)
    u.encode(t, k, n, ln)
    t[G // 2, k + 3, 100] ^= 1
    r = bench.verify_slice(u, synth, torch, t, pres, g0, G)
    assert r["ok"] is False and not r["parity_match"] and r["decode_match"], r
