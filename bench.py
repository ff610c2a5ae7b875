"""bench.py -- device-resident RS(20,10) encode + decode throughput on MI355X.

One step = one pass of the hot path over one batch per GPU (BASELINE.json
configs[1] + configs[2]): rs_encode2 of G groups (RS(20,10), 1250-B shards)
followed by rs_decode2 of the same G groups with 5 random erasures each
(decode plans built on the GPU inside the step).  Inputs are resident in HBM
before the timed region.  Groups are sharded across ranks with no data-path
collective (weak scaling by default: G groups per GPU; --scaling strong
splits --total-groups, C4's 2^20, across the ranks).

Prints ONE JSON line (rank 0).  value = payload GiB/s over all GPUs, payload
= k*len bytes per group per operation (encode + decode).  roofline is for the
dominant kernel (encode), measured with HIP events on the launch stream;
cpu_baseline times the reference codec (oracle/_ref) -- or the C restatement
if the reference build is absent -- on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident RS encode+decode GiB/s (payload bytes) & FEC-groups/s, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
K, M, LEN, STRIDE, ERASURES = 20, 10, 1250, 1280, 5


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--groups", type=int, default=65536, help="groups per GPU (weak scaling)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    p.add_argument("--total-groups", type=int, default=1 << 20, help="strong scaling total (C4)")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip the C2-worst / C3 lines")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    p.add_argument("--share-device", action="store_true",
                   help="map every rank to cuda:0 (rehearsing N>1 on a 1-GPU box, gloo only)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="per-launch HBM bytes from a rocprofv3 --pmc pass (optional)")
    return p.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import udpspeeder_amd as u
    from udpspeeder_amd import shard, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(args.backend, rank=rank, world_size=world)

    if args.scaling == "weak":
        g0, g1 = shard.weak_range(rank, args.groups)
    else:
        g0, g1 = shard.strong_range(rank, world, args.total_groups)
    G = g1 - g0
    n = K + M

    # ---- inputs resident in HBM before timing
    buf = torch.empty((G, n, STRIDE), dtype=torch.uint8, device=dev)
    u.fill_data(buf, K, LEN, synth.DATA_SEED, g0=g0)
    present = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, g0, G, n, ERASURES)).to(dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    u.reserve(K, n, G, stream)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        u.encode(buf, K, n, LEN, stream=stream)
        if i is not None:
            ev[i][1].record(stream)
        u.decode(buf, present, K, n, LEN, status=status, stream=stream)
        if i is not None:
            ev[i][2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        # max over ranks: the job is as slow as its slowest GPU
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    bad = int((status != 0).sum().item())
    enc_ms = statistics.mean(a.elapsed_time(b) for a, b, _ in ev)
    dec_ms = statistics.mean(b.elapsed_time(c) for _, b, c in ev)

    total_groups = G * world if args.scaling == "weak" else args.total_groups
    payload = 2.0 * total_groups * K * LEN * args.steps  # encode + decode
    value = payload / elapsed / 2**30
    groups_per_s = total_groups * args.steps / elapsed

    # ---- roofline for the dominant kernel (encode): algorithmic bytes / launch
    alg_bytes = G * (K + M) * LEN  # read k*len + write m*len per group
    achieved = alg_bytes / (enc_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("groups") == G and tj.get("kernel"):
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "encode RS(20,10)", "alg_bytes_per_launch": alg_bytes,
                "avg_launch_ms": round(enc_ms, 4)}
    # decode roofline: k*len read + e*len written for every group with e > 0
    pres_np = present.cpu().numpy()
    e_rows = (pres_np[:, :K] == 0).sum(1)
    dec_alg = int(((e_rows > 0) * K * LEN).sum() + (e_rows * LEN).sum())
    dec_achieved = dec_alg / (dec_ms * 1e-3) / 1e9
    roofline_decode = {"bound": "hbm", "achieved": round(dec_achieved, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(dec_achieved / HBM_PEAK_GBS, 4),
                       "kernel": "fused decode RS(20,10), 5 random erasures",
                       "alg_bytes_per_launch": dec_alg, "avg_launch_ms": round(dec_ms, 4)}
    extras = None
    if rank == 0 and world == 1 and not args.no_extras:
        extras = extra_configs(u, synth, torch, dev, buf, G)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(buf, present, G, args.cpu_threads)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: SplitMix64 payload bytes, seeded 5-of-30 erasures per group",
            "config": {"workload": "C1+C2: RS(20,10) encode + decode (5 random erasures), "
                                   "1250-B shards, device-resident",
                       "k": K, "m": M, "len": LEN, "shard_stride": STRIDE,
                       "groups_per_gpu": G, "global_groups": total_groups,
                       "parallelism": f"groups sharded over {world} GPU(s), no collective"},
            "groups_per_s": round(groups_per_s, 1),
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
            "decode_failures": bad,
            "roofline": roofline,
            "roofline_decode": roofline_decode,
            "cpu_baseline": cpu,
            "other_configs": extras,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _time_ms(torch, fn, reps=10, warm=2):
    import statistics as st
    ts = []
    for i in range(reps + warm):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if i >= warm:
            ts.append(a.elapsed_time(b))
    return st.median(ts)


def extra_configs(u, synth, torch, dev, buf, G):
    """BASELINE configs beside the headline step (device-resident, N=1):
    C2 worst case (5 data erasures) and C3 (ragged mode-0 mix)."""
    n = K + M
    out = {}
    # C2 worst case: every group loses 5 data shards
    pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED + 1, 0, G, n, ERASURES,
                                                  limit=K)).to(dev)
    st = torch.empty(G, dtype=torch.int32, device=dev)
    ms = _time_ms(torch, lambda: u.decode(buf, pres, K, n, LEN, status=st))
    alg = G * (K + ERASURES) * LEN
    out["c2_worst_5_data_erasures"] = {
        "decode_ms": round(ms, 4), "groups": G,
        "payload_GiBps": round(G * K * LEN / (ms * 1e-3) / 2**30, 1),
        "alg_GBps": round(alg / (ms * 1e-3) / 1e9, 1), "failures": int((st != 0).sum().item())}
    # C3: ragged mix from -f 1:3,2:4,10:6,20:10, len 64..1250, one bucketed launch
    table = u.rs_from_str(synth.C3_FEC)
    ks, ms_, ls = synth.ragged_mix(synth.RAGGED_SEED, 0, G, [y for _, y in table])
    groups, total = u.make_groups(ks, ks + ms_, ls)
    base = torch.zeros(total, dtype=torch.uint8, device=dev)
    dg = u.rs.groups_to_device(groups, dev)
    u.rs.fill_ragged(base, dg, G, synth.DATA_SEED)
    plan = u.rs.RaggedPlan(groups)
    t = _time_ms(torch, lambda: plan.encode(base))
    alg = int(((ks + ms_) * ls).sum())
    out["c3_ragged_encode"] = {
        "encode_ms": round(t, 4), "groups": G, "bitslice_plan": plan.bitslice,
        "payload_GiBps": round(float((ks * ls).sum()) / (t * 1e-3) / 2**30, 1),
        "alg_GBps": round(alg / (t * 1e-3) / 1e9, 1), "alg_bytes": alg,
        "roofline_frac": round(alg / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    plan.close()
    del base
    # f2: cook + de_cook of every packet C1 emits (8-B header + 1250-B shard)
    from udpspeeder_amd.cook import CookContext
    plen, pstride = 8 + LEN, 1312
    npk = G * n
    pk = torch.empty((npk, pstride), dtype=torch.uint8, device=dev)
    pk[:, :8] = 0x5A
    pk.view(G, n, pstride)[:, :, 8:8 + LEN] = buf[:, :, :LEN]
    lens = torch.full((npk,), plen, dtype=torch.int32, device=dev)
    olen = torch.empty_like(lens)
    back = torch.empty_like(lens)
    ctx = CookContext(b"bench-key", 0)
    tcs, tds = [], []
    for i in range(6):  # refill, cook, de_cook: the round trip must restore the packets
        pk.view(G, n, pstride)[:, :, 8:8 + LEN] = buf[:, :, :LEN]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        ctx.cook(pk, lens, cap=pstride, out_len=olen, seed=7 + i)
        e[1].record()
        ctx.decook(pk, olen, cap=pstride, out_len=back)
        e[2].record()
        torch.cuda.synchronize()
        if i:
            tcs.append(e[0].elapsed_time(e[1]))
            tds.append(e[1].elapsed_time(e[2]))
    tc, td = statistics.median(tcs), statistics.median(tds)
    ok = bool((back == plen).all()) and torch.equal(
        pk.view(G, n, pstride)[:, :, 8:8 + LEN], buf[:, :, :LEN])
    cooked = float(olen.float().mean())
    alg = npk * (plen + cooked)
    out["f2_cook_decook"] = {
        "packets": npk, "len": plen, "key": True, "cook_ms": round(tc, 4),
        "decook_ms": round(td, 4), "cook_Mpps": round(npk / tc / 1e3, 1),
        "decook_Mpps": round(npk / td / 1e3, 1),
        "cook_frac": round(alg / (tc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "decook_frac": round(alg / (td * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "roundtrip_ok": ok}
    ctx.close()
    del pk
    return out


def cpu_baseline(buf, present, G, threads):
    """Time the reference codec (oracle/_ref/libref_rs.so: lib/fec.cpp + lib/rs.cpp
    unmodified) on this host -- or the C restatement if the reference build is
    absent -- on the same C1+C2 groups; median of 3 reps; checked against the
    GPU's parity."""
    import numpy as np
    import platform
    from oracle.cpu import Oracle, Reference

    nthreads = threads or min(16, os.cpu_count() or 1)
    n = K + M
    host = buf.cpu().numpy()  # data + GPU parity (+ decoded rows == data)
    pres = present.cpu().numpy()
    sample = min(G, 65536)
    gpu_par = host[:sample, K:, :LEN].copy()
    if Reference.available():
        lib, kind = Reference(), "reference"
        enc = lambda b: lib.encode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample,
                                         nthreads)
        dec = lambda b: lib.decode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample,
                                         pres[:sample], False, nthreads)
    else:
        lib, kind = Oracle(), "port"
        nthreads = 1
        enc = lambda b: lib.encode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample)
        dec = lambda b: lib.decode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample,
                                         pres[:sample])
    pristine = np.ascontiguousarray(host[:sample])
    times = []
    for _ in range(3):
        b = pristine.copy()
        b[:, K:] = 0
        t0 = time.perf_counter()
        enc(b)
        t1 = time.perf_counter()
        if _ == 0 and not (b[:, K:, :LEN] == gpu_par).all():
            raise SystemExit("cpu_baseline: CPU parity differs from GPU parity")
        t2 = time.perf_counter()
        dec(b)
        t3 = time.perf_counter()
        times.append((t1 - t0) + (t3 - t2))
    med = statistics.median(times)
    gib = 2.0 * sample * K * LEN / med / 2**30
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                 if l.startswith("model name")][0]
    except (OSError, IndexError):
        model = platform.processor()
    return {"value": round(gib, 3), "unit": "GiB/s", "cores": nthreads, "kind": kind,
            "sample": f"{sample} groups RS(20,10)x1250B encode + decode(5 erasures), "
                      f"median of 3 reps, {nthreads} threads on {model}",
            "groups_per_s": round(sample / med, 1)}


if __name__ == "__main__":
    main()
