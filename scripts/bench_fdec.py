"""Time the batched FEC receive side on one GPU.

Workload: the packets of one connection's mode-0 stream (1200-byte payloads,
-f 20:10, mtu 1250: RS(20,10) groups of 1203-byte shards), framed on the GPU by
FecEncoder, with ERASE of every group's 30 packets dropped (seeded), in one
batch into FecDecoder.  Reports the host plan, the device run (gather + decode
+ pack + D2H of the data rows, HIP events) and the host output resolution.

    python scripts/bench_fdec.py [--groups 65536] [--erase 5] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from udpspeeder_amd.fec import SLOT_PACKET, FecDecoder, FecEncoder  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--erase", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=100000, help="0 = no CPU baseline")
    args = ap.parse_args()
    plen = 1200 if args.mode == 0 else 1250
    npk = args.groups * 20
    dev = torch.device("cuda:0")
    lens_in = np.full(npk, plen, np.int32)
    offs_in = np.arange(npk, dtype=np.uint64) * np.uint64(1216)
    inbuf = torch.randint(0, 256, (int(offs_in[-1]) + plen + 64,), dtype=torch.uint8, device=dev)
    enc = FecEncoder("20:10", args.mode, 1250, 200, seq0=1)
    p = enc.plan(lens_in, offs_in, inbuf)
    S = FecEncoder.slot_stride_for(int(p.groups["fec_len"].max()))
    slots = torch.empty(p.n_slots * S, dtype=torch.uint8, device=dev)
    enc.run(slots, S)
    torch.cuda.synchronize()
    pk = p.packets
    # drop `erase` of each group's packets (groups are runs of equal headers' seq)
    rng = np.random.default_rng(7)
    host_all = slots.cpu().numpy()
    g0 = p.groups["slot0"]
    n_g = (p.groups["k"] + p.groups["m"]).astype(np.int64)
    assert (n_g == n_g[0]).all()
    dropped = np.zeros(p.n_slots, bool)
    pick = np.argsort(rng.random((len(g0), int(n_g[0]))), axis=1)[:, :args.erase]
    dropped[(g0[:, None] + pick).ravel()] = True
    keep = ~dropped[pk["slot"]]
    kept = pk[keep]
    offs = (kept["slot"].astype(np.uint64) * np.uint64(S) + np.uint64(SLOT_PACKET))
    lens = kept["len"].astype(np.int32)
    res = []
    outs = 0
    dec = FecDecoder()  # steady state: one manager, a fresh seq range every rep
    oi = offs.astype(np.int64)
    seq0 = (host_all[oi].astype(np.uint32) << 24 | host_all[oi + 1].astype(np.uint32) << 16 |
            host_all[oi + 2].astype(np.uint32) << 8 | host_all[oi + 3].astype(np.uint32))
    for rep in range(args.reps + 1):
        if rep:  # new sequence numbers (the anti-replay window has seen the old ones)
            sq = seq0 + np.uint32(rep * 1_000_003)
            for b in range(4):
                host_all[oi + b] = (sq >> np.uint32(24 - 8 * b)).astype(np.uint8)
            slots.copy_(torch.from_numpy(host_all))
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        dp = dec.plan(host_all, lens, offs, slots)
        t1 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dec.run()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        n_out = len(dec.outputs_raw()[1])  # C++ resolution; no Python bytes copies
        t3 = time.perf_counter()
        if rep:
            res.append((t1 - t0, e0.elapsed_time(e1), t3 - t2))
        outs = n_out
    med = lambda i: float(np.median([r[i] for r in res]))
    payload = int(npk) * plen
    cpu = None
    if args.cpu_sample:
        # the reference's fec_decode_manager_t (oracle/_ref) on one thread -- its
        # libev thread -- over the first packets of the same stream
        from oracle.fec_frame import FecReference
        if FecReference.available():
            n = min(args.cpu_sample, len(lens))
            chan = [host_all[int(oi[i]):int(oi[i]) + int(lens[i])].tobytes() for i in range(n)]
            t0 = time.perf_counter()
            _, rout, _ = FecReference().decode(chan)
            dt = time.perf_counter() - t0
            cpu = {"kind": "reference", "threads": 1, "sample_packets": n,
                   "packets_in_per_s": round(n / dt, 1), "outputs": len(rout),
                   "note": "includes the driver's copy of each packet in and out"}
    print(json.dumps({
        "cpu_baseline": cpu,
        "mode": args.mode, "groups": int(len(g0)), "packets_in": int(len(kept)),
        "erased_per_group": args.erase, "decoded_groups": int(dp.n_decodes), "outputs": outs,
        "plan_ms": round(med(0) * 1e3, 3), "run_ms": round(med(1), 4),
        "outputs_ms": round(med(2) * 1e3, 3),
        "run_payload_GBps": round(payload / (med(1) * 1e-3) / 1e9, 1),
        "run_Mpps_in": round(len(kept) / med(1) / 1e3, 1)}))


if __name__ == "__main__":
    main()
