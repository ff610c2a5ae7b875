"""CPU: synthetic-workload definitions (product side) agree with the oracle's,
and the multi-rank group partition is disjoint and complete (gloo, world 2)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from udpspeeder_amd import synth, shard
from oracle import cpu


def test_erasures_match_oracle():
    a = synth.erasure_present(synth.ERASE_SEED, 5, 300, 30, 5)
    b = cpu.present_from_erasures(cpu.erasures(cpu.ERASE_SEED, 5, 300, 30, 5), 30)
    assert (a == b).all() and (a.sum(1) == 25).all()
    a = synth.erasure_present(7, 0, 50, 30, 5, limit=20)
    assert (a[:, 20:] == 1).all()


def test_ragged_matches_oracle(golden):
    ty = np.array([y for _, y in golden.mats["c3_table"].tolist()])
    k1, m1, l1 = synth.ragged_mix(synth.RAGGED_SEED, 0, 65536, ty)
    k2, m2, l2 = cpu.ragged_draw(cpu.RAGGED_SEED, 0, 65536, ty)
    assert (k1 == k2).all() and (m1 == m2).all() and (l1 == l2).all()
    assert int((k1 * l1).sum()) == golden.full["c3_ragged_encode"]["sum_payload"]


def test_ranges():
    assert shard.weak_range(3, 100) == (300, 400)
    rs = [shard.strong_range(r, 8, 1 << 20) for r in range(8)]
    assert rs[0][0] == 0 and rs[-1][1] == 1 << 20
    assert all(rs[i][1] == rs[i + 1][0] for i in range(7))
    w = np.random.default_rng(1).integers(1, 1000, 1000)
    br = shard.balanced_ranges(w, 4)
    assert br[0][0] == 0 and br[-1][1] == 1000
    sums = [w[a:b].sum() for a, b in br]
    assert max(sums) - min(sums) <= 2 * w.max()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g0, g1 = shard.strong_range(rank, world, 1000)
    owned = torch.zeros(1000, dtype=torch.int32)
    owned[g0:g1] = 1
    dist.all_reduce(owned)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench's max-over-ranks timing
    if rank == 0:
        q.put((owned.min().item(), owned.max().item(), t.item()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_partition():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert all(p.exitcode == 0 for p in ps)
    lo, hi, tmax = q.get(timeout=5)
    assert lo == 1 and hi == 1 and tmax == 2.0


def test_ragged_erasures_match_oracle():
    rng = np.random.default_rng(4)
    ks = rng.integers(1, 60, 3000)
    ms = rng.integers(0, 40, 3000)
    ms[:5] = [0, 1, 2, 3, 4]
    a = synth.ragged_erasures(synth.ERASE_SEED, 7, ks + ms, ms, 5)
    b = cpu.ragged_erasures(cpu.ERASE_SEED, 7, ks + ms, ms, 5)
    assert (a == b).all()
    assert ((a.sum(1)) == ks + ms - np.minimum(ms, 5)).all()
    bits = synth.present_bits(a)
    assert bits.dtype == np.uint32 and bits.shape == (3000, 8)
    back = np.unpackbits(bits.view(np.uint8), axis=1, bitorder="little")
    assert (back == a).all()


def test_group_hashes_restatement_agrees():
    """bench.py's per-group checksum (synth.group_hashes_dev, torch) and the
    checker's numpy restatement (oracle.cpu.group_hashes) agree bit for bit on
    strided slices of a [G, n, stride] batch, and a one-byte change moves the
    group's checksum."""
    import torch
    from oracle.cpu import group_hashes
    from udpspeeder_amd import synth
    b = np.random.default_rng(9).integers(0, 256, (300, 30, 1280), dtype=np.uint8)
    t = torch.from_numpy(b)
    for sl in ((slice(None), slice(20, None), slice(0, 1250)),
               (slice(None), slice(0, 20), slice(0, 1250)), (slice(5, 77), slice(3, 4), slice(0, 17))):
        assert (synth.group_hashes_dev(t[sl], chunk=64) == group_hashes(b[sl])).all()
    h0 = group_hashes(b[:, 20:, :1250])
    b[7, 25, 1000] ^= 0x80
    h1 = group_hashes(b[:, 20:, :1250])
    assert (h0 != h1).sum() == 1 and h0[7] != h1[7]
    assert synth.hashes_digest(h0) != synth.hashes_digest(h1)


def test_c4_fixture_covers_every_bench_range(golden):
    """tests/golden/full_hashes.json holds reference digests for every group
    range a bench.py rank owns: strong splits of 2^20 over 1/2/4/8 ranks and
    the weak 65,536-group blocks (so a driver N-GPU run checks all its ranks)."""
    from udpspeeder_amd import shard
    R = golden.full["c4_rank_slices"]["ranges"]
    for w in (1, 2, 4, 8):
        for r in range(w):
            g0, g1 = shard.strong_range(r, w, 1 << 20)
            assert f"{g0}-{g1}" in R
        for r in range(w):
            g0, g1 = shard.weak_range(r, 65536)
            assert f"{g0}-{g1}" in R
