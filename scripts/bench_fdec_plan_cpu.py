"""Receive-side planner cost on the host alone (no GPU): rsmi_fdec_plan on a
plan-only decoder over bench_pipeline.py's stream shape -- mode 0, RS(20,10)
groups of 1203-byte shards, 5 of every 30 packets lost, ~41 K packets per
batch.  Payload bytes are zeros (the planner reads headers only).

    python scripts/bench_fdec_plan_cpu.py [--batches 12] [--per-batch 40960]
"""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from udpspeeder_amd import lib  # noqa: E402
from udpspeeder_amd._lib import check  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--per-batch", type=int, default=40960)
    ap.add_argument("--shard", type=int, default=1203)
    ap.add_argument("--dense", action="store_true", help="headers 16 B apart (cache-resident input)")
    args = ap.parse_args()
    k, m, L = 20, 10, args.shard
    ngroups = args.batches * args.per_batch // (k + m - 5) + 1
    rng = np.random.default_rng(7)
    keep = np.ones((ngroups, k + m), bool)
    pick = np.argsort(rng.random((ngroups, k + m)), axis=1)[:, :5]
    np.put_along_axis(keep, pick, False, axis=1)
    gi, idx = np.nonzero(keep)
    npk = len(gi)
    stride = 16 if args.dense else 8 + L + 5  # header + shard, padded
    buf = np.zeros(npk * stride, np.uint8)
    rec = buf.reshape(npk, stride)
    seq = (gi + 1).astype(np.uint32)
    rec[:, 0:4] = seq.astype(">u4").view(np.uint8).reshape(npk, 4)
    rec[:, 4] = 0
    rec[:, 5] = k
    rec[:, 6] = m
    rec[:, 7] = idx
    lens = np.full(npk, 8 + L, np.int32)
    offs = np.arange(npk, dtype=np.uint64) * np.uint64(stride)
    L_ = lib()
    h = C.c_void_p()
    check(L_.rsmi_fdec_create(0, C.byref(h)), "create")
    per = npk // args.batches
    ret = np.zeros(per + 1, np.int32)
    nd = C.c_int64()
    times = []
    for b in range(args.batches):
        sl = slice(b * per, (b + 1) * per)
        ln, of = np.ascontiguousarray(lens[sl]), np.ascontiguousarray(offs[sl])
        t = time.perf_counter()
        check(L_.rsmi_fdec_plan(h, per, ln.ctypes.data, of.ctypes.data, buf.ctypes.data, None, 0,
                                ret.ctypes.data, C.byref(nd)), "plan")
        times.append(time.perf_counter() - t)
    L_.rsmi_fdec_destroy(h)
    t = sorted(times[2:])
    med = t[len(t) // 2]
    print(f"{per} packets per batch, {nd.value} decodes: plan median {med * 1e3:.3f} ms "
          f"({per / med / 1e6:.1f} Mpps, {med / per * 1e9:.1f} ns/packet)")


if __name__ == "__main__":
    main()
