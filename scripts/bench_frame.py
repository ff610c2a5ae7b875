"""Time the batched FEC framing on one GPU.

Workload: one connection's packets through fec_encode_manager_t semantics in one
batch -- mode 0 (blob) with 1200-byte packets under -f 20:10, mtu 1250 (20
packets per blob, RS(20,10) groups of 1203-byte shards), or mode 1 with
1250-byte packets (RS(20,10), 1252-byte shards).  Reports the host planning
time, the frame kernel (blob assembly + headers), the encode launches and the
carry copy, each from HIP events on the launch stream, with the frame kernel's
algorithmic bytes (payload read + k*fec_len shard bytes and n headers written).

    python scripts/bench_frame.py [--mode 0] [--groups 65536] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from udpspeeder_amd.fec import FecEncoder  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--len", type=int, default=0, help="packet bytes (default 1200 / 1250)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fec", default="20:10")
    args = ap.parse_args()
    plen = args.len or (1200 if args.mode == 0 else 1250)
    npk = args.groups * 20
    lens = np.full(npk, plen, np.int32)
    offs = (np.arange(npk, dtype=np.uint64) * np.uint64((plen + 15) // 16 * 16))
    dev = torch.device("cuda:0")
    inbuf = torch.randint(0, 256, (int(offs[-1]) + plen + 64,), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    res = []
    for rep in range(args.reps + 1):
        enc = FecEncoder(args.fec, args.mode, 1250, 200, seq0=rep)
        t0 = time.perf_counter()
        p = enc.plan(lens, offs, inbuf)
        t_plan = time.perf_counter() - t0
        S = FecEncoder.slot_stride_for(int(p.groups["fec_len"].max()))
        slots = torch.empty(p.n_slots * S, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        enc.run(slots, S)
        e1.record(s)
        torch.cuda.synchronize()
        if rep:
            res.append((t_plan, e0.elapsed_time(e1)))
        g = p.groups
        enc.close()
        del slots
    t_plan = float(np.median([r[0] for r in res]))
    t_run = float(np.median([r[1] for r in res]))
    ng = len(g["k"])
    kk, mm, fl = g["k"].astype(np.int64), g["m"].astype(np.int64), g["fec_len"].astype(np.int64)
    payload = int(lens.sum())
    frame_bytes = payload + int((kk * fl).sum()) + 8 * int((kk + mm).sum())
    enc_bytes = int(((kk + mm) * fl).sum())
    print(json.dumps({
        "mode": args.mode, "packets": npk, "packet_len": plen, "groups": ng,
        "k": int(np.median(kk)), "m": int(np.median(mm)), "fec_len": int(np.median(fl)),
        "emitted_packets": int(len(p.packets)), "plan_ms": round(t_plan * 1e3, 3),
        "run_ms": round(t_run, 4), "run_Mpps_in": round(npk / t_run / 1e3, 1),
        "payload_GBps": round(payload / (t_run * 1e-3) / 1e9, 1),
        "frame_alg_bytes": frame_bytes, "encode_alg_bytes": enc_bytes,
        "run_alg_GBps": round((frame_bytes + enc_bytes) / (t_run * 1e-3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
