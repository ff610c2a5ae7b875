"""Time the cook / de_cook kernels on framed FEC packets.

Workload: every packet RS(20,10) emits for G groups -- 8-byte header + 1250-byte
shard = 1258-byte packets, n = 30 per group -- in 1312-byte slots, cooked with
device-drawn IVs under a key, then de_cooked.  Prints one JSON line.

The CPU baseline is the reference's own do_cook / de_cook (oracle/_ref,
packet.cpp compiled unmodified) on a bounded sample of the same packets:
do_cook on one thread (its IV PRNG is a process global), de_cook on
--cpu-threads threads.

    python scripts/bench_cook.py [--groups 65536] [--iters 20] [--cpu-sample 200000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from udpspeeder_amd.cook import CookContext  # noqa: E402

HBM_PEAK_GBS = 8000.0


def cpu_baseline(args, host, olen):
    from oracle.cpu import CookReference
    if not CookReference.available():
        return None
    ref = CookReference()
    ref.config(args.key.encode(), args.flags)
    n = min(args.cpu_sample, host.shape[0])
    plain = np.zeros((n, args.stride), np.uint8)
    plain[:, :args.len] = host[:n, :args.len]
    lens = np.full(n, args.len, np.int32)
    b = plain.copy()
    t0 = time.perf_counter()
    out = ref.cook_batch(b, args.stride, lens)
    tc = time.perf_counter() - t0
    thr = args.cpu_threads or min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    back = ref.decook_batch(b, args.stride, out, thr)
    td = time.perf_counter() - t0
    assert (back == args.len).all() and (b[:, :args.len] == plain[:, :args.len]).all()
    model = ""
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                 if l.startswith("model name")][0]
    except (OSError, IndexError):
        pass
    return {"kind": "reference", "sample_packets": n, "cpu": model,
            "cook_Mpps": round(n / tc / 1e6, 3), "cook_threads": 1,
            "decook_Mpps": round(n / td / 1e6, 3), "decook_threads": thr}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--len", type=int, default=1258)
    ap.add_argument("--stride", type=int, default=1312)
    ap.add_argument("--key", default="bench-key")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=200000, help="0 = no CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    npk = args.groups * 30
    buf = torch.randint(0, 256, (npk, args.stride), dtype=torch.uint8, device=dev)
    orig = buf[:, :args.len].clone()
    lens = torch.full((npk,), args.len, dtype=torch.int32, device=dev)
    out = torch.empty_like(lens)
    back = torch.empty_like(lens)
    ctx = CookContext(args.key.encode(), args.flags)
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tc = td = 0.0
    for it in range(args.iters + 2):
        e[0].record(s)
        ctx.cook(buf, lens, cap=args.stride, out_len=out, seed=it)
        e[1].record(s)
        ctx.decook(buf, out, cap=args.stride, out_len=back)
        e[2].record(s)
        torch.cuda.synchronize()
        if it >= 2:
            tc += e[0].elapsed_time(e[1])
            td += e[1].elapsed_time(e[2])
    assert bool((back == args.len).all()) and torch.equal(buf[:, :args.len], orig)
    tc /= args.iters
    td /= args.iters
    olen = float(out.float().mean())
    # algorithmic bytes: cook reads len, writes the cooked packet; de_cook reads
    # the cooked packet, writes len
    cb = npk * (args.len + olen)
    line = {
        "packets": npk, "len": args.len, "mean_cooked_len": round(olen, 2),
        "cook_ms": round(tc, 4), "decook_ms": round(td, 4),
        "cook_GBps": round(cb / tc / 1e6, 1), "decook_GBps": round(cb / td / 1e6, 1),
        "cook_frac": round(cb / tc / 1e6 / HBM_PEAK_GBS, 4),
        "decook_frac": round(cb / td / 1e6 / HBM_PEAK_GBS, 4),
        "cook_Mpps": round(npk / tc / 1e3, 1), "decook_Mpps": round(npk / td / 1e3, 1),
        "key": args.key, "flags": args.flags}
    if args.cpu_sample:
        line["cpu_baseline"] = cpu_baseline(args, orig.cpu().numpy(), olen)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
