"""Time the batched FEC framing on one GPU.

Workload: one connection's packets through fec_encode_manager_t semantics in one
batch -- mode 0 (blob) with 1200-byte packets under -f 20:10, mtu 1250 (20
packets per blob, RS(20,10) groups of 1203-byte shards), or mode 1 with
1250-byte packets (RS(20,10), 1252-byte shards).  One encoder in steady state
(state carries from batch to batch).  Reports the host planning time and the
device run (plan upload, frame kernel, encode launches, carry copy; HIP events
on the launch stream), with the frame kernel's algorithmic bytes (payload read
+ k*fec_len shard bytes and 8-byte headers written).

The CPU baseline is the reference's own fec_encode_manager_t (oracle/_ref,
fec_manager.cpp compiled unmodified) on one thread -- the reference runs it on
its single libev thread -- over a bounded sample of the same events.

With --cook the run also cooks every emitted packet (do_cook, key set,
device-drawn IVs): "dev" -- rsmi_fenc_run_cooked_dev into a device buffer;
"host" -- the same into pinned host memory (the cook's stores are the D2H
transfer, packets land where sendmmsg reads them); "sep" -- the unfused
pipeline it replaces: run_dev, in-place rsmi_cook_dev, then a D2H copy.

    python scripts/bench_frame.py [--mode 0] [--groups 65536] [--reps 5] [--cook dev|host|sep]
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


def cpu_baseline(args, plen, sample):
    from oracle.fec_frame import FecReference
    if not FecReference.available():
        return None
    fr = FecReference()
    fr.config(args.fec, args.mode, 1250, 200)
    rng = np.random.default_rng(3)
    ev = [rng.integers(0, 256, plen, dtype=np.uint8).tobytes() for _ in range(sample)]
    t0 = time.perf_counter()
    _, pk, _ = fr.encode(ev)
    dt = time.perf_counter() - t0
    return {"kind": "reference", "threads": 1, "sample_packets": sample,
            "packets_in_per_s": round(sample / dt, 1), "packets_out": len(pk),
            "note": "includes the driver's copy of each output packet"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--len", type=int, default=0, help="packet bytes (default 1200 / 1250)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fec", default="20:10")
    ap.add_argument("--cpu-sample", type=int, default=100000, help="0 = no CPU baseline")
    ap.add_argument("--cook", default="", choices=["", "dev", "host", "sep"])
    ap.add_argument("--cook-flags", type=int, default=0, help="RSMI_COOK_NO_* flags (measurement: 1 = no CRC)")
    args = ap.parse_args()
    plen = args.len or (1200 if args.mode == 0 else 1250)
    npk = args.groups * 20
    lens = np.full(npk, plen, np.int32)
    offs = (np.arange(npk, dtype=np.uint64) * np.uint64((plen + 15) // 16 * 16))
    dev = torch.device("cuda:0")
    inbuf = torch.randint(0, 256, (int(offs[-1]) + plen + 64,), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    res = []
    enc = FecEncoder(args.fec, args.mode, 1250, 200, seq0=1)  # steady state: one manager
    slots = out = None
    ctx = None
    if args.cook:
        from udpspeeder_amd.cook import CookContext
        ctx = CookContext(b"passwd123", args.cook_flags)
    for rep in range(args.reps + 1):
        t0 = time.perf_counter()
        p = enc.plan(lens, offs, inbuf)
        t_plan = time.perf_counter() - t0
        S = FecEncoder.slot_stride_for(int(p.groups["fec_len"].max()))
        if slots is None or slots.numel() < p.n_slots * S:
            slots = torch.empty(p.n_slots * S, dtype=torch.uint8, device=dev)
            if args.cook:
                out = torch.empty(p.n_slots * S, dtype=torch.uint8)
                out = out.cuda() if args.cook == "dev" else out.pin_memory()
        if args.cook == "sep":
            offs_d = torch.from_numpy(p.packets["slot"].astype(np.int64) * S + 120).to(dev)
            lens_d = torch.from_numpy(p.packets["len"].astype(np.int32)).to(dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        tc = time.perf_counter()
        if args.cook in ("dev", "host"):
            enc.run_cooked(slots, S, ctx, rep + 1, out=out)
        else:
            enc.run(slots, S)
            if args.cook == "sep":
                ctx.cook(slots, lens_d, cap=S - 120, offsets=offs_d, seed=rep + 1)
                out[:p.n_slots * S].copy_(slots[:p.n_slots * S], non_blocking=True)
        e1.record(s)
        tc = time.perf_counter() - tc
        torch.cuda.synchronize()
        if rep:
            res.append((t_plan, e0.elapsed_time(e1), tc))
        g = p.groups
    t_plan = float(np.median([r[0] for r in res]))
    t_run = float(np.median([r[1] for r in res]))
    t_call = float(np.median([r[2] for r in res]))
    ng = len(g["k"])
    kk, mm, fl = g["k"].astype(np.int64), g["m"].astype(np.int64), g["fec_len"].astype(np.int64)
    payload = int(lens.sum())
    frame_bytes = payload + int((kk * fl).sum()) + 8 * int((kk + mm).sum())
    enc_bytes = int(((kk + mm) * fl).sum())
    line = {
        "mode": args.mode, "packets": npk, "packet_len": plen, "groups": ng,
        "k": int(np.median(kk)), "m": int(np.median(mm)), "fec_len": int(np.median(fl)),
        "emitted_packets": int(len(p.packets)), "plan_ms": round(t_plan * 1e3, 3),
        "run_ms": round(t_run, 4), "call_host_ms": round(t_call * 1e3, 4), "run_Mpps_in": round(npk / t_run / 1e3, 1),
        "payload_GBps": round(payload / (t_run * 1e-3) / 1e9, 1),
        "frame_alg_bytes": frame_bytes, "encode_alg_bytes": enc_bytes,
        "run_alg_GBps": round((frame_bytes + enc_bytes) / (t_run * 1e-3) / 1e9, 1)}
    if args.cook:
        line["cook"] = {"dev": "fused, device out", "host": "fused, pinned host out (cook = D2H)",
                        "sep": "run_dev + in-place cook + D2H copy"}[args.cook]
        line["cooked_packets_per_s"] = round(len(p.packets) / (t_run * 1e-3), 1)
        line["cooked_wire_GBps"] = round(int(p.packets["len"].sum() + 23 * len(p.packets)) /
                                         (t_run * 1e-3) / 1e9, 1)
    if args.cpu_sample:
        line["cpu_baseline"] = cpu_baseline(args, plen, args.cpu_sample)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
