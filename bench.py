"""bench.py -- device-resident RS(20,10) encode + decode throughput on MI355X.

One step = one pass of the hot path over one batch per GPU: rs_encode2 of the
rank's groups (RS(20,10), 1250-B shards) followed by rs_decode2 of the same
groups with 5 random erasures each (decode plans built on the GPU inside the
step).  Inputs are resident in HBM before the timed region.

* N = 1 (default): BASELINE configs[1] + configs[2], 65,536 groups.
* N > 1: configs[4] (C4), 2^20 groups split into contiguous ranges over the
  ranks (strong scaling), one process per GPU, no data-path collective: FEC
  groups are independent.  ``--scaling weak`` keeps
  ``--groups`` per GPU instead.

``python bench.py --gpus N`` without a torch.distributed launcher starts the N
ranks itself (``torch.distributed.run`` on 127.0.0.1) before touching the
GPU; a WORLD_SIZE that disagrees with --gpus is an error.

Prints ONE JSON line (rank 0).  value = payload GiB/s over all GPUs (k*len
bytes per group per operation, encode + decode), timed between barriers and
taken as the max over ranks.  ``roofline`` is for whichever kernel takes
longer per step, measured with HIP events on the launch stream;
``cpu_baseline`` times the reference codec (oracle/_ref) on this host, 1
thread and one thread per CPU of the process's affinity set (16 beside it).
After the timed region every rank checks its own slice's bytes against the
reference's digests (``parity_ok``, one entry per rank).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident RS encode+decode GiB/s (payload bytes) & FEC-groups/s, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
K, M, LEN, STRIDE, ERASURES = 20, 10, 1250, 1280, 5
C4_GROUPS = 1 << 20
SETTLE_EXTRA_MS = 150.0  # untimed calls before each other_configs measurement (clock ramp)
TRAFFIC = {"encode": os.path.join(ROOT, "profiles", "traffic.json"),
           "decode": os.path.join(ROOT, "profiles", "traffic_decode.json")}
# The sources a kernel's counters depend on: a traffic JSON carries their
# digest from the counter pass (scripts/pmc_traffic.py), and roofline() reports
# its bytes only while the sources are unchanged.
KERNEL_SOURCES = {"encode": ["udpspeeder_amd/csrc/bitslice.hip", "udpspeeder_amd/csrc/bitslice_kern.hpp",
                             "udpspeeder_amd/csrc/gen_bitslice.py"],
                  "decode": ["udpspeeder_amd/csrc/decode.hip", "udpspeeder_amd/csrc/lagrange.hpp"]}


def kernel_source_sha(which):
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES[which]:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--settle-ms", type=float, default=400.0,
                   help="untimed steps for at least this long before the --warmup steps: the GPU "
                        "clocks ramp over the first tens of ms of load, and the VALU-heavy decode "
                        "runs ~15%% slower until they have (never part of the timed region)")
    p.add_argument("--groups", type=int, default=65536, help="groups per GPU (weak scaling)")
    p.add_argument("--scaling", choices=["weak", "strong"], default=None,
                   help="default: weak at N=1 (C1+C2), strong over --total-groups at N>1 (C4)")
    p.add_argument("--total-groups", type=int, default=C4_GROUPS, help="strong scaling total")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="threads of the all-cores CPU leg (default: len(os.sched_getaffinity(0)), "
                        "the CPUs this process may run on; a 16-thread leg is reported beside it)")
    p.add_argument("--no-verify", action="store_true",
                   help="skip the after-the-timed-region check of every rank's bytes")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip the other_configs lines")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    p.add_argument("--share-device", action="store_true",
                   help="map every rank to cuda:0 (rehearsing N>1 on a 1-GPU box, gloo only)")
    p.add_argument("--workload", choices=["c1c2", "c3"], default="c1c2",
                   help="c1c2 (default): RS(20,10) encode + decode (C1+C2 at N=1, C4 at N>1); c3: "
                        "the ragged mode-0 mix (k 1..20, -f 1:3,2:4,10:6,20:10, len 64..1250), "
                        "--total-groups of it split over the ranks by balanced (k+m)*len ranges")
    p.add_argument("--rehearse", action="store_true",
                   help="CPU only: run the launcher / barrier / max-over-ranks / JSON path with a "
                        "numpy stand-in step (tests; never a measurement)")
    return p.parse_args(argv)


def launch_ranks(args) -> int:
    """Start args.gpus ranks through torch.distributed.run and return its exit
    code.  Runs before this process touches the GPU."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}")
    scaling = args.scaling or ("weak" if world == 1 else "strong")
    if args.rehearse:
        return rehearse(args, world, rank, scaling)

    import numpy as np
    import torch
    import torch.distributed as dist

    import udpspeeder_amd as u
    from udpspeeder_amd import shard, synth

    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(args.backend, rank=rank, world_size=world)

    if args.workload == "c3":
        return run_c3(args, world, rank, dev, scaling)

    if scaling == "weak":
        g0, g1 = shard.weak_range(rank, args.groups)
        total_groups = args.groups * world
    else:
        g0, g1 = shard.strong_range(rank, world, args.total_groups)
        total_groups = args.total_groups
    G = g1 - g0
    n = K + M

    # ---- inputs resident in HBM before timing
    buf = torch.empty((G, n, STRIDE), dtype=torch.uint8, device=dev)
    u.fill_data(buf, K, LEN, synth.DATA_SEED, g0=g0)
    present = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, g0, G, n, ERASURES)).to(dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    u.reserve(K, n, G, stream)

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        u.encode(buf, K, n, LEN, stream=stream)
        if i is not None:
            ev[i][1].record(stream)
        # rebuilt rows in their own slots.  The reference's placement
        # (rows over the parity survivors, lib/fec.cpp:872-877, and rs_decode's
        # pointer permutation as a slot map) decodes as fast but makes this
        # step's next encode 2.6 % slower (it overwrites the lines the decode
        # just wrote; profiles/r06/place_step_ab.txt); verify_slice checks both
        u.decode(buf, present, K, n, LEN, status=status, stream=stream)
        if i is not None:
            ev[i][2].record(stream)

    # settle: untimed steps until the clocks have ramped (see --settle-ms)
    t_settle = time.perf_counter()
    settle_steps = 0
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for _ in range(8):
            step()
        settle_steps += 8
        torch.cuda.synchronize()
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
    enc_ms = statistics.mean(a.elapsed_time(b) for a, b, _ in ev)
    dec_ms = statistics.mean(b.elapsed_time(c) for _, b, c in ev)
    bad = int((status != 0).sum().item())
    extras = None
    copy_peak = None
    if rank == 0 and world == 1 and not args.no_extras:
        extras = extra_configs(u, synth, torch, dev, buf, G)
        copy_peak = hbm_copy_peak(u, torch, dev)
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, every N
        cpu = cpu_baseline(buf, present, G, args.cpu_threads)
    # after the timed region (and after the lines above, which read buf's
    # parity): this rank's bytes against the reference's digests
    check = None if args.no_verify else verify_slice(u, synth, torch, buf, present, g0, G)
    ok_flags = [-1.0] * world
    ok_flags[rank] = -1.0 if check is None or check.get("ok") is None else float(check["ok"])
    parity_ok = [None if f < 0 else bool(f) for f in ok_flags]
    if world > 1:
        # max over ranks: the job is as slow as its slowest GPU; every rank's
        # parity flag rides along in its own slot (-1 elsewhere)
        t = torch.tensor([elapsed, enc_ms, dec_ms, float(bad)] + ok_flags, dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, enc_ms, dec_ms, bad = float(t[0]), float(t[1]), float(t[2]), int(t[3])
        parity_ok = [None if float(f) < 0 else bool(f > 0.5) for f in t[4:]]

    payload_op = float(total_groups) * K * LEN  # one operation over the whole job
    value = 2.0 * payload_op * args.steps / elapsed / 2**30
    groups_per_s = total_groups * args.steps / elapsed

    # ---- rooflines: algorithmic bytes per launch / average launch time
    enc_alg = G * (K + M) * LEN  # read k*len + write m*len per group
    pres_np = present.cpu().numpy()
    e_rows = (pres_np[:, :K] == 0).sum(1)
    dec_alg = int(((e_rows > 0) * K * LEN).sum() + (e_rows * LEN).sum())  # k*len read + e*len written
    roof = {
        "encode": roofline("encode", "k_bs2_20_30: split-k bit-sliced RS(20,10) encode", enc_alg, enc_ms, G),
        "decode": roofline("decode", "k_decode_fused: RS(20,10) decode, 5 random erasures",
                           dec_alg, dec_ms, G),
    }
    dominant = "decode" if dec_ms >= enc_ms else "encode"
    other = "encode" if dominant == "decode" else "decode"

    if rank == 0:
        if scaling == "weak":
            workload = ("C1+C2: RS(20,10) encode + decode (5 random erasures), 1250-B shards, "
                        "device-resident" if world == 1 else
                        f"weak scaling: {G} groups per GPU, RS(20,10) encode + decode")
        else:
            workload = (f"C4: RS(20,10) encode + decode (5 random erasures), 1250-B shards, "
                        f"{total_groups} groups split over {world} GPU(s), device-resident")
        if copy_peak:
            for which, r in roof.items():  # the same achieved rate against the measured copy / mix
                r["frac_of_copy_peak"] = round(r["achieved"] / copy_peak["GBps"], 4)
                mix = copy_peak["mixes_GBps"]["2:1 (encode)" if which == "encode" else "6:1 (decode)"]
                r["frac_of_mix_peak"] = round(r["achieved"] / mix, 4)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "settle": {"ms": args.settle_ms, "steps": settle_steps},
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: SplitMix64 payload bytes, seeded 5-of-30 erasures per group",
            "config": {"workload": workload, "k": K, "m": M, "len": LEN, "shard_stride": STRIDE,
                       "groups_per_gpu": G, "global_groups": total_groups,
                       "parallelism": f"groups sharded over {world} GPU(s), no collective"},
            "groups_per_s": round(groups_per_s, 1),
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
            "encode_GiBps": round(payload_op / (enc_ms * 1e-3) / 2**30, 2),
            "decode_GiBps": round(payload_op / (dec_ms * 1e-3) / 2**30, 2),
            "decode_failures": bad,
            "parity_ok": parity_ok,
            "parity_check": None if check is None else {
                k_: v for k_, v in check.items() if k_ != "ok"},
            "roofline": roof[dominant],
            f"roofline_{other}": roof[other],
            "hbm_copy_peak": copy_peak,
            "cpu_baseline": cpu,
            "other_configs": extras,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_c3(args, world, rank, dev, scaling):
    """--workload c3: the ragged mode-0 mix (BASELINE configs[3]) as the step.
    The mix of --total-groups groups (strong) or --groups per rank (weak) is
    drawn per group id (synth.ragged_mix, so every rank sees the same mix),
    and ranks own contiguous ranges of near-equal (k+m)*len
    (shard.balanced_ranges) -- no collective on the data path.  A step is one
    bucketed encode launch of the rank's groups and one ragged decode of them
    with min(5, m) erasures each.  After the timed region each rank checks its
    slice: the parity of 256 sampled groups against the oracle, and that the
    decode restored every erased row; rank 0 times the reference codec on a
    bounded sample of its groups (1 thread, one rs_encode2 / rs_decode2 per
    group, as the reference calls them)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import udpspeeder_amd as u
    from udpspeeder_amd import shard, synth

    table = u.rs_from_str(synth.C3_FEC)
    ty = [y for _, y in table]
    if scaling == "weak":
        g0, g1 = shard.weak_range(rank, args.groups)
        total = args.groups * world
    else:
        total = args.total_groups
        ka, ma, la = synth.ragged_mix(synth.RAGGED_SEED, 0, total, ty)
        g0, g1 = shard.balanced_ranges((ka + ma) * la, world)[rank]
    G = g1 - g0
    ks, ms_, ls = synth.ragged_mix(synth.RAGGED_SEED, g0, G, ty)
    groups, nbytes = u.make_groups(ks, ks + ms_, ls)
    base = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    dg = u.rs.groups_to_device(groups, dev)
    u.rs.fill_ragged(base, dg, G, synth.DATA_SEED, g0=g0)
    for kk in sorted(set(zip(ks.tolist(), (ks + ms_).tolist()))):
        u.prepare_code(*kk)
    plan = u.rs.RaggedPlan(groups)
    flags = synth.ragged_erasures(synth.ERASE_SEED, g0, ks + ms_, ms_, ERASURES)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(dev)
    status = torch.empty(G, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        plan.encode(base)
        if i is not None:
            ev[i][1].record(stream)
        plan.decode(base, bits, status=status)  # own slots, as the C2 step
        if i is not None:
            ev[i][2].record(stream)

    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
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
    enc_ms = statistics.mean(a.elapsed_time(b) for a, b, _ in ev)
    dec_ms = statistics.mean(b.elapsed_time(c) for _, b, c in ev)
    bad = int((status != 0).sum().item())
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = c3_cpu_baseline(u, base, groups, ks, ms_, ls, flags)
    ok = None
    if not args.no_verify:
        ok = c3_verify(u, synth, torch, base, groups, ks, ms_, ls, g0, plan, bits, status)
    payload = float((ks * ls).sum())
    flag = -1.0 if ok is None else float(ok)
    t = torch.tensor([elapsed, enc_ms, dec_ms, float(bad)] + [flag if r == rank else -1.0 for r in range(world)]
                     + [payload if r == rank else 0.0 for r in range(world)], dtype=torch.float64,
                     device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        # max over ranks for the times; per-rank slots for the flags and payloads
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, enc_ms, dec_ms, bad = float(t[0]), float(t[1]), float(t[2]), int(t[3])
    parity_ok = [None if float(f) < 0 else bool(f > 0.5) for f in t[4:4 + world]]
    job_payload = float(t[4 + world:].sum())
    e = ((flags[:, :20] == 0) & (np.arange(20)[None, :] < ks[:, None])).sum(1)
    enc_alg = int(((ks + ms_) * ls).sum())
    dec_alg = int((((e > 0) * ks + e) * ls).sum())
    roof = {"encode": roofline("encode", "k_bs_ragged: C3 bucketed bit-sliced encode", enc_alg, enc_ms, -1),
            "decode": roofline("decode", "k_decode_ragged_mix: C3 ragged decode", dec_alg, dec_ms, -1)}
    dominant = "decode" if dec_ms >= enc_ms else "encode"
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(2.0 * job_payload * args.steps / elapsed / 2**30, 2),
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: SplitMix64 payload bytes, per-group (k, m, len) draws, min(5, m) erasures",
            "config": {"workload": f"C3: ragged mode-0 mix -f {synth.C3_FEC}, len 64..1250, {total} groups "
                                   f"over {world} GPU(s) by balanced (k+m)*len ranges, device-resident",
                       "groups_rank0": G, "global_groups": total,
                       "parallelism": f"groups sharded over {world} GPU(s), no collective"},
            "groups_per_s": round(total * args.steps / elapsed, 1),
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4), "decode_failures": bad,
            "parity_ok": parity_ok,
            "parity_check": "per rank: parity of 256 sampled groups vs the oracle; every erased row "
                            "restored by the decode",
            "roofline": roof[dominant], f"roofline_{'encode' if dominant == 'decode' else 'decode'}":
                roof["encode" if dominant == "decode" else "decode"],
            "cpu_baseline": cpu}), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


def c3_verify(u, synth, torch, base, groups, ks, ms_, ls, g0, plan, bits, status):
    """The rank's C3 slice after the timed loop: 256 sampled groups' parity
    equal the oracle's (the C restatement of lib/rs.cpp, pinned to the
    reference's vectors), and a decode of the slice with every erased slot
    poisoned restores the data rows (the step decoded a codeword)."""
    import numpy as np
    from oracle.cpu import Oracle
    o = Oracle()
    host = base.cpu().numpy()
    G = len(ks)
    rng = np.random.default_rng(g0)
    ok = True
    for g in rng.choice(G, min(256, G), replace=False):
        k, n, ln = int(ks[g]), int(ks[g] + ms_[g]), int(ls[g])
        off, ss = int(groups[g].offset), int(groups[g].shard_stride)
        one = np.zeros(n * ss, np.uint8)
        one[:k * ss] = host[off:off + k * ss]
        o.encode_batch(k, n, one, n * ss, ss, ln, 1)
        ok &= bool((one[k * ss:].reshape(n - k, ss)[:, :ln] ==
                    host[off + k * ss:off + n * ss].reshape(n - k, ss)[:, :ln]).all())
    data = [host[int(groups[g].offset):int(groups[g].offset) + int(ks[g]) * int(groups[g].shard_stride)].copy()
            for g in range(G)]
    flags = synth.ragged_erasures(synth.ERASE_SEED, g0, ks + ms_, ms_, ERASURES)
    for g in range(G):  # poison the erased slots
        off, ss = int(groups[g].offset), int(groups[g].shard_stride)
        for j in np.nonzero(flags[g, :int(ks[g] + ms_[g])] == 0)[0]:
            host[off + j * ss:off + (j + 1) * ss] = 0xA5
    poisoned = torch.from_numpy(host)
    base.copy_(poisoned)
    plan.decode(base, bits, status=status)  # the step's call: rows in their own slots
    torch.cuda.synchronize()
    out = base.cpu().numpy()
    ok &= int((status != 0).sum().item()) == 0
    for g in range(G):
        off, ss, k, ln = int(groups[g].offset), int(groups[g].shard_stride), int(ks[g]), int(ls[g])
        got = out[off:off + k * ss].reshape(k, ss)[:, :ln]
        ok &= bool((got == data[g].reshape(k, ss)[:, :ln]).all())
        if not ok:
            return ok
    # the reference's placement on the same input: each data[i] read through
    # the slot map (rs_decode's pointer permutation)
    base.copy_(poisoned)
    smap = torch.empty((G, 20), dtype=torch.uint8, device=base.device)
    plan.decode(base, bits, status=status, placement="reference", slot_map=smap)
    torch.cuda.synchronize()
    out = base.cpu().numpy()
    m = smap.cpu().numpy()
    ok &= int((status != 0).sum().item()) == 0
    for g in range(G):
        off, ss, k, ln, n = (int(groups[g].offset), int(groups[g].shard_stride), int(ks[g]), int(ls[g]),
                             int(ks[g] + ms_[g]))
        got = out[off:off + n * ss].reshape(n, ss)[m[g, :k].astype(np.int64), :ln]
        ok &= bool((got == data[g].reshape(k, ss)[:, :ln]).all())
        if not ok:
            break
    return ok


def c3_cpu_baseline(u, base, groups, ks, ms_, ls, flags, sample=4096, reps=3):
    """The reference codec (oracle/_ref: lib/fec.cpp + lib/rs.cpp unmodified)
    on the first `sample` groups of this rank's C3 slice: one rs_encode2 and
    one rs_decode2-equivalent call per group (its own k, n, len), 1 thread,
    median of `reps`; payload GiB/s as the GPU line (k*len per operation)."""
    import numpy as np
    from oracle.cpu import Oracle, Reference
    ref = Reference.available()
    lib = Reference() if ref else Oracle()
    host = base.cpu().numpy()
    S = min(sample, len(ks))
    spans = [(int(groups[g].offset), int(groups[g].shard_stride), int(ks[g]), int(ks[g] + ms_[g]), int(ls[g]))
             for g in range(S)]
    if ref:  # get_code is lazy and not thread-safe: build every code first (lib/rs.cpp:42-55)
        for k, n in sorted({(k, n) for _, _, k, n, _ in spans}):
            lib.lib.ref_prewarm(k, n)
    tot = []
    for _ in range(reps):
        bufs = [host[off:off + n * ss].copy() for off, ss, k, n, ln in spans]
        for b, (off, ss, k, n, ln) in zip(bufs, spans):
            b[k * ss:] = 0
        t0 = time.perf_counter()
        for g, (b, (off, ss, k, n, ln)) in enumerate(zip(bufs, spans)):
            lib.encode_batch(k, n, b, n * ss, ss, ln, 1)
            lib.decode_batch(k, n, b, n * ss, ss, ln, 1, np.ascontiguousarray(flags[g, :n]).reshape(1, n))
        tot.append(time.perf_counter() - t0)
    pay = float(sum(k * ln for _, _, k, _, ln in spans))
    return {"value": round(2.0 * pay / statistics.median(tot) / 2**30, 3), "unit": "GiB/s", "cores": 1,
            "kind": "reference" if ref else "port",
            "sample": f"first {S} groups of rank 0's C3 slice, one encode + one decode call per group "
                      f"(Python loop over ctypes calls included), median of {reps}"}


def verify_slice(u, synth, torch, buf, present, g0, G):
    """This rank's bytes, checked after the timed region against digests the
    real reference produced (tests/golden/full_hashes.json, c4_rank_slices
    ranges, made by oracle/gen_golden.py --c4) for exactly this group range:
    * parity: the timed loop's encode output (the parity rows now in buf);
    * decode: the rank's slice refilled as the non-codeword input (data from
      DATA_SEED, parity from DATA_SEED ^ 0xFFFF), every erased slot poisoned,
      one decode through the same call as the step, the k data rows compared
      (pins which survivors rs_decode uses, lib/rs.cpp:24-39); then the same
      input again through the reference's placement (rows over the parity
      survivors), its rows read through the slot map and the map compared
      with the host closed form (rs_decode's pointer permutation).
    Digests are sha256 over per-group checksums (synth.group_hashes_dev), so
    8 B per group leave the device.  ``ok`` is None when no fixture covers the
    range (e.g. a --groups the fixtures were not made for)."""
    t0 = time.perf_counter()
    path = os.path.join(ROOT, "tests", "golden", "full_hashes.json")
    try:
        F = json.load(open(path))["c4_rank_slices"]
        R = F["ranges"].get(f"{g0}-{g0 + G}")
    except (OSError, ValueError, KeyError):
        F, R = None, None
    if R is None:
        return {"ok": None, "range": [g0, g0 + G], "why": "no reference digest for this range"}
    n = K + M
    par = synth.hashes_digest(synth.group_hashes_dev(buf[:, K:, :LEN]))
    def refill():
        u.fill_data(buf, K, LEN, F["seed"], g0=g0)
        u.fill_data(buf[:, K:], M, LEN, F["parity_seed"], g0=g0)
        buf.masked_fill_((present == 0).unsqueeze(-1), 0xA5)  # erased slots hold junk

    refill()
    st = u.decode(buf, present, K, n, LEN)
    fails = int((st != 0).sum().item())
    dat_own = synth.hashes_digest(synth.group_hashes_dev(buf[:, :K, :LEN]))
    refill()
    smap = torch.empty((G, K), dtype=torch.uint8, device=buf.device)
    st = u.decode(buf, present, K, n, LEN, placement="reference", slot_map=smap)
    fails += int((st != 0).sum().item())
    # the data rows read through the slot map, in data[] order (the pointer
    # permutation rs_decode leaves the caller), and the map itself against the
    # host closed form on a sample of groups
    map_ok = all((smap[g].cpu().numpy() == u.ref_slot_map(K, n, present[g].cpu().numpy())).all()
                 for g in range(0, G, max(1, G // 64)))
    dat = synth.hashes_digest(synth.group_hashes_dev(u.reference_rows(buf, smap)[:, :, :LEN]))
    ok = (par == R["parity_gsum"] and dat_own == R["data_out_gsum"] and dat == R["data_out_gsum"]
          and fails == 0 and map_ok)
    return {"ok": ok, "range": [g0, g0 + G], "parity_match": par == R["parity_gsum"],
            "decode_match": dat_own == R["data_out_gsum"], "ref_placement_decode_match": dat == R["data_out_gsum"],
            "slot_map_match": map_ok,
            "decode_failures": fails,
            "check_s": round(time.perf_counter() - t0, 2),
            "what": "reference digests of this rank's encode parity and non-codeword decode"}


def hbm_copy_peak(u, torch, dev, nbytes=2 << 30, reps=8):
    """SURVEY 8(d)'s second reference line: a measured device-to-device copy
    of 2 GiB on this box (read + written bytes / time, median of `reps` after
    2 warm), the best of librsmi's copy kernel (`rsmi_copy_peak`, 4 or 8
    16-byte words per thread, plain or nontemporal) and torch's `copy_`,
    each variant's rate listed."""
    from udpspeeder_amd._lib import check
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(7)
    L = u.lib()

    def rate(fn):
        ts = []
        for i in range(reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(e0.elapsed_time(e1))
        return round(2 * nbytes / (statistics.median(ts) * 1e-3) / 1e9, 1)

    names = ["rsmi_u4", "rsmi_u8", "rsmi_u4_nt", "rsmi_u8_nt"]
    got = {}
    for v, name in enumerate(names):
        # (torch's current stream: the events above are recorded on it)
        got[name] = rate(lambda: check(L.rsmi_copy_peak(b.data_ptr(), a.data_ptr(), nbytes, v,
                                                        torch.cuda.current_stream().cuda_stream),
                                       "rsmi_copy_peak"))
    assert torch.equal(a[:1 << 20], b[:1 << 20]) and torch.equal(a[-(1 << 20):], b[-(1 << 20):])
    got["torch_copy_"] = rate(lambda: b.copy_(a))
    # read:write mixes of the codec kernels (rsmi_copy_peak variants 4-6):
    # bytes read + written per second
    a.random_(0, 256)
    nr = nbytes // (16 * 256 * 24) * (16 * 256 * 24)
    mixes = {}
    for v, name, wfrac in [(4, "read_only", 0.0), (5, "2:1 (encode)", 0.5), (6, "6:1 (decode)", 1 / 6)]:
        r = rate(lambda: check(L.rsmi_copy_peak(b.data_ptr(), a.data_ptr(), nr, v,
                                                torch.cuda.current_stream().cuda_stream), "rsmi_copy_peak"))
        mixes[name] = round(r / 2 * nr * (1 + wfrac) / nbytes, 1)  # rate() counted 2 * nbytes
    del a, b
    best = max(got, key=got.get)
    return {"GBps": got[best], "best": best, "variants_GBps": got, "bytes_each_way": nbytes,
            "mixes_GBps": mixes,
            "how": "device-to-device copy of 2 GiB (read + write bytes / time), median of 8 after 2 warm, "
                   "best variant; mixes: the same for kernels that read 2 GiB and write none, half, a sixth"}


def roofline(which, kernel, alg_bytes, ms, G):
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    traffic, note = None, "no counter pass for this kernel and size"
    path = TRAFFIC[which]
    if os.path.exists(path):
        try:
            tj = json.load(open(path))
            # only counters of the kernel this build launches, from its current sources
            if tj.get("groups") == G and kernel.split(":")[0] == tj.get("kernel"):
                if tj.get("source_sha256") == kernel_source_sha(which):
                    traffic = tj.get("hbm_bytes_per_launch")
                    note = f"PMC pass {os.path.relpath(path, ROOT)} (sources unchanged since)"
                else:
                    note = "stale: the kernel's sources changed since the counter pass"
        except (OSError, ValueError):
            traffic = None
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": note,
            "kernel": kernel, "alg_bytes_per_launch": int(alg_bytes), "avg_launch_ms": round(ms, 4)}


def rehearse(args, world, rank, scaling):
    """The multi-rank harness without a GPU (tests only): gloo, a numpy XOR
    stand-in for the step, the same barriers, max-over-ranks and JSON line."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from udpspeeder_amd import shard
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    total = args.total_groups if scaling == "strong" else args.groups * world
    g0, g1 = (shard.strong_range(rank, world, total) if scaling == "strong"
              else shard.weak_range(rank, args.groups))
    a = np.random.default_rng(rank).integers(0, 256, (g1 - g0, 64), dtype=np.uint8)
    for _ in range(args.warmup):
        a ^= a[::-1]
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a ^= a[::-1]
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    owned = torch.tensor([float(g1 - g0)], dtype=torch.float64)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.all_reduce(owned)
    if rank == 0:
        print(json.dumps({"metric": "rehearsal (no GPU): harness only", "rehearsal": True,
                          "value": round(float(owned.item()) * args.steps / elapsed, 1),
                          "unit": "groups/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "scaling": scaling,
                          "groups_covered": int(owned.item()), "global_groups": total}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def _time_ms(torch, fn, reps=10, warm=2, spread=None):
    """Median per-call GPU time of fn, calls enqueued back to back.  With a
    synchronise before every call, the start event would fire on an idle GPU
    while the host is still in fn's launch path (~0.1 ms of Python and HIP
    calls), and that gap would be counted as kernel time.  The warm calls run
    for at least SETTLE_EXTRA_MS, so the clocks are up again after the host
    work between configs (see --settle-ms)."""
    t0 = time.perf_counter()
    i = 0
    while i < warm or (time.perf_counter() - t0) * 1e3 < SETTLE_EXTRA_MS:
        fn()
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps + 1)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) for a, b in ev[1:]]  # the first call waits on the host
    if spread is not None:  # min / max per-call time: how far one box's reps scatter
        spread["spread_ms"] = [round(min(ts), 4), round(max(ts), 4)]
    return statistics.median(ts)


def extra_configs(u, synth, torch, dev, buf, G):
    """BASELINE configs beside the headline step (device-resident, N=1):
    C2 worst case (5 data erasures), C3 (ragged mode-0 mix), C4's 2^20 groups
    on this one GPU (the strong-scaling base), the f2 cook/de_cook row and the
    per-call latency of the level-1 drop-in (rs_encode2 / rs_decode2)."""
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
        "alg_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
        "roofline_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "failures": int((st != 0).sum().item())}
    out.update(c3_configs(u, synth, torch, dev, G))
    out["c4_one_gpu"] = c4_one_gpu(u, synth, torch, dev)
    out["rtc_f10_5_encode"] = rtc_config(u, synth, torch, dev)
    out["f2_cook_decook"] = cook_config(torch, dev, buf, G)
    out["f1_f2_frame_encode_cook"] = frame_cook_config(torch, dev)
    # the other setting of RSMI_OPT_PARITY_COOK (the parity cooked in the
    # encoder's epilogue), same workload
    from udpspeeder_amd._lib import RSMI_OPT_PARITY_COOK
    cur = u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, 0)
    u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, cur)
    alt = frame_cook_config(torch, dev, parity_cook=not cur)
    out["f1_f2_frame_encode_cook"]["parity_cook_option"] = bool(cur)
    out["f1_f2_frame_encode_cook"]["other_setting"] = {
        "parity_cook_option": not cur, "run_ms": alt["run_ms"], "parity_cook_runs": alt["parity_cook_runs"],
        "lengths_ok": alt.get("lengths_ok")}
    out["f1_collector_200_connections"] = collector_config(torch, dev)
    out["dropin_latency_us"] = dropin_latency_both(u)
    return out


def c3_configs(u, synth, torch, dev, G):
    """C3: ragged mix from -f 1:3,2:4,10:6,20:10, len 64..1250: one bucketed
    encode launch, then one ragged decode launch with min(5, m) random
    erasures per group (synth.ragged_erasures) on the encoded batch."""
    import numpy as np
    out = {}
    table = u.rs_from_str(synth.C3_FEC)
    ks, ms_, ls = synth.ragged_mix(synth.RAGGED_SEED, 0, G, [y for _, y in table])
    groups, total = u.make_groups(ks, ks + ms_, ls)
    base = torch.zeros(total, dtype=torch.uint8, device=dev)
    dg = u.rs.groups_to_device(groups, dev)
    u.rs.fill_ragged(base, dg, G, synth.DATA_SEED)
    plan = u.rs.RaggedPlan(groups)
    sp_e, sp_d = {}, {}
    t = _time_ms(torch, lambda: plan.encode(base), spread=sp_e)
    alg = int(((ks + ms_) * ls).sum())
    out["c3_ragged_encode"] = {
        "encode_ms": round(t, 4), **sp_e, "groups": G, "bitslice_plan": plan.bitslice,
        "payload_GiBps": round(float((ks * ls).sum()) / (t * 1e-3) / 2**30, 1),
        "alg_GBps": round(alg / (t * 1e-3) / 1e9, 1), "alg_bytes": alg,
        "roofline_frac": round(alg / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    flags = synth.ragged_erasures(synth.ERASE_SEED, 0, ks + ms_, ms_, ERASURES)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(dev)
    st = torch.empty(G, dtype=torch.int32, device=dev)
    t = _time_ms(torch, lambda: plan.decode(base, bits, status=st), spread=sp_d)
    e = ((flags[:, :20] == 0) & (np.arange(20)[None, :] < ks[:, None])).sum(1)
    alg = int((((e > 0) * ks + e) * ls).sum())  # k*len read + e*len written, groups with e > 0
    out["c3_ragged_decode"] = {
        "decode_ms": round(t, 4), **sp_d, "groups": G, "rebuilt_rows": int(e.sum()),
        "payload_GiBps": round(float((ks * ls).sum()) / (t * 1e-3) / 2**30, 1),
        "alg_GBps": round(alg / (t * 1e-3) / 1e9, 1), "alg_bytes": alg,
        "roofline_frac": round(alg / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "failures": int((st != 0).sum().item())}
    plan.close()
    del base
    return out


def rtc_config(u, synth, torch, dev, k=10, m=5, groups=131072):
    """-f 10:5, a code with no build-time network: RS(10,15) over 1250-B shards,
    131072 groups (C1's data volume), through the network librsmi compiled at
    run time (hipRTC), and through the generic table kernel for comparison."""
    from udpspeeder_amd._lib import ENC_BITSLICE_RTC
    n = k + m
    t0 = time.time()
    u.wait_code(k, n)
    compile_s = time.time() - t0
    kind = u.code_encoder(k, n)
    buf = torch.zeros((groups, n, 1280), dtype=torch.uint8, device=dev)
    u.fill_data(buf, k, LEN, synth.DATA_SEED)
    ms = _time_ms(torch, lambda: u.encode(buf, k, n, LEN))
    last = u.lib().rsmi_last_encoder()
    prev = u.rs.set_bitslice(False)
    try:
        ms_generic = _time_ms(torch, lambda: u.encode(buf, k, n, LEN), reps=5)
    finally:
        u.rs.set_bitslice(prev)
    del buf
    alg = groups * n * LEN
    return {"code": f"{k}:{m}", "groups": groups, "len": LEN,
            "encoder": "bitslice_rtc" if kind == ENC_BITSLICE_RTC and last == kind else
                       f"kind{kind}/ran{last}",
            "wait_code_s": round(compile_s, 2), "encode_ms": round(ms, 4),
            "alg_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
            "roofline_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "generic_encode_ms": round(ms_generic, 4),
            "generic_roofline_frac": round(alg / (ms_generic * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def c4_one_gpu(u, synth, torch, dev, steps=5):
    """C4's 2^20 RS(20,10) groups on one GPU: the base of the strong-scaling
    curve that bench.py --gpus N (N > 1) measures."""
    n = K + M
    Gc = C4_GROUPS
    b = torch.empty((Gc, n, STRIDE), dtype=torch.uint8, device=dev)
    u.fill_data(b, K, LEN, synth.DATA_SEED)
    p = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, 0, Gc, n, ERASURES)).to(dev)
    st = torch.empty(Gc, dtype=torch.int32, device=dev)
    u.reserve(K, n, Gc)

    def step():
        u.encode(b, K, n, LEN)
        u.decode(b, p, K, n, LEN, status=st)
    ms = _time_ms(torch, step, reps=steps, warm=1)
    r = {"groups": Gc, "ms_per_step": round(ms, 3),
         "GiBps": round(2.0 * Gc * K * LEN / (ms * 1e-3) / 2**30, 1),
         "failures": int((st != 0).sum().item())}
    del b
    return r


def cook_config(torch, dev, buf, G):
    """f2: cook + de_cook of every packet C1 emits (8-B header + 1250-B shard)."""
    from udpspeeder_amd.cook import CookContext
    n = K + M
    plen, pstride = 8 + LEN, 1312
    npk = G * n
    pk = torch.empty((npk, pstride), dtype=torch.uint8, device=dev)
    pk[:, :8] = 0x5A
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
    alg = npk * (plen + cooked)  # read the plain packet, write the cooked one
    ctx.close()
    del pk
    return {"packets": npk, "len": plen, "key": True, "cook_ms": round(tc, 4),
            "decook_ms": round(td, 4), "cook_Mpps": round(npk / tc / 1e3, 1),
            "decook_Mpps": round(npk / td / 1e3, 1), "alg_bytes": int(alg),
            "cook_frac": round(alg / (tc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "decook_frac": round(alg / (td * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "roundtrip_ok": ok}


def frame_cook_config(torch, dev, groups=65536, reps=4, parity_cook=None):
    """f1 + f2 fused: one connection's 1200-B datagrams (mode 0, -f 20:10, mtu
    1250: 65,536 RS(20,10) groups) through rsmi_fenc_run_cooked_dev -- framing,
    bit-sliced encode and do_cook of every emitted packet in one run into a
    device buffer.  Planning is host work outside the timed region (bench_frame.py
    times it); each rep plans the next batch of the same stream."""
    import numpy as np
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecEncoder
    import udpspeeder_amd as u
    from udpspeeder_amd._lib import RSMI_OPT_PARITY_COOK
    prev = None if parity_cook is None else u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, int(parity_cook))
    plen = 1200
    npk = groups * 20
    lens = np.full(npk, plen, np.int32)
    offs = np.arange(npk, dtype=np.uint64) * np.uint64(1216)
    inbuf = torch.randint(0, 256, (npk * 1216 + 64,), dtype=torch.uint8, device=dev)
    enc = FecEncoder("20:10", 0, 1250, 200, seq0=1)
    ctx = CookContext(b"bench-key")
    slots = out = None
    ts, nout, ok, epi = [], 0, True, 0
    for i in range(reps + 1):
        p = enc.plan(lens, offs, inbuf)
        S = FecEncoder.slot_stride_for(int(p.groups["fec_len"].max()))
        if slots is None or slots.numel() < p.n_slots * S:  # a batch may open more slots (carry)
            slots = out = None
            slots = torch.empty(p.n_slots * S + 64 * S, dtype=torch.uint8, device=dev)
            out = torch.empty_like(slots)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ol = enc.run_cooked(slots, S, ctx, 11 + i, out=out)
        e1.record()
        torch.cuda.synchronize()
        nout = len(p.packets)
        ok = ok and bool((ol[:nout] > torch.from_numpy(p.packets["len"]).to(dev)).all())
        epi = enc.last_parity_cooked()
        if i:
            ts.append(e0.elapsed_time(e1))
    t = statistics.median(ts)
    enc.close()
    ctx.close()
    if prev is not None:
        u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, prev)
    del slots, out, inbuf
    return {"datagrams_in": npk, "datagram_len": plen, "groups": groups, "packets_out": nout,
            "run_ms": round(t, 4), "parity_cook_runs": epi, "datagrams_in_per_s": round(npk / (t * 1e-3), 1),
            "cooked_packets_per_s": round(nout / (t * 1e-3), 1),
            "what": "rsmi_fenc_run_cooked_dev: plan upload (groups, packet runs; source records "
                    "read in place) + k_expand_packets + k_cook_frame (data packets framed into "
                    "their slots and cooked in one pass) + k_bs2_20_30 + carry + k_cook of the "
                    "parity packets; device-resident, key on, device-drawn IVs", "lengths_ok": ok}


def collector_config(torch, dev, ncon=200, flushes=12, seed=5):
    """The cross-connection collector (rsmi_fenc_run_many): 200 connections
    (max_conn_num, common.h:112), each with its own fec_encode_manager_t
    (-f 20:10, mode 0, mtu 1250; connection.h:244-245), each flushing 64-256
    datagrams of 64-1200 B per 8 ms timer tick (fec_manager.h:30, the timer's
    input(0, 0) included).  One flush = plan every manager on the host, then
    the byte work: framing + encode + do_cook into device memory, either as
    ONE collector launch set or as 200 rsmi_fenc_run_cooked_dev calls.
    Reports the GPU time of the run part (HIP events, per flush, median) and
    the wall time of the whole flush including the host planning: the
    collector plans every manager in one native call (rsmi_fenc_plan_many, a
    pool of host threads), the per-connection mode one FecEncoder.plan each."""
    import numpy as np
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecCollector, FecEncoder
    rng = np.random.default_rng(seed)
    ctx = CookContext(b"bench-key")
    res = {}
    for mode in ("collector", "per_connection"):
        encs = [FecEncoder("20:10", 0, 1250, 200, seq0=i * 7919) for i in range(ncon)]
        col = FecCollector() if mode == "collector" else None
        S = FecEncoder.slot_stride_for(1250)
        slots = out = None
        gpu_ms, wall_ms, plan_ms, npk_tot, nev_tot = [], [], [], 0, 0
        r2 = np.random.default_rng(seed)  # the same traffic for both modes
        for f in range(flushes):
            nper = r2.integers(64, 257, ncon)
            lens = [np.concatenate([r2.integers(64, 1201, n), [-1]]).astype(np.int32) for n in nper]
            tot = int(sum(int(np.maximum(l, 0).sum()) for l in lens))
            inbuf = torch.randint(0, 256, (tot + 64,), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "collector":  # every manager planned by one native call (host threads)
                flat = np.concatenate(lens)
                offs_flat = np.zeros(flat.size, np.uint64)
                np.cumsum(np.maximum(flat[:-1], 0), out=offs_flat[1:])
                cuts = np.cumsum([0] + [len(l) for l in lens])
                ns_, npk_, _ = col.plan_many(encs, [flat[cuts[i]:cuts[i + 1]] for i in range(ncon)],
                                             [offs_flat[cuts[i]:cuts[i + 1]] for i in range(ncon)], inbuf)
                nsl, npk = int(ns_.sum()), int(npk_.sum())
                plans = [type("P", (), {"n_slots": int(x)}) for x in ns_]
            else:
                o, plans = 0, []
                for ci in range(ncon):
                    l = lens[ci]
                    offs = np.concatenate([[0], np.cumsum(np.maximum(l, 0))[:-1]]).astype(np.uint64) + np.uint64(o)
                    o += int(np.maximum(l, 0).sum())
                    plans.append(encs[ci].plan(l, offs, inbuf))
                nsl = sum(p.n_slots for p in plans)
                npk = sum(len(p.packets) for p in plans)
            t_plan = time.perf_counter()
            if slots is None or slots.numel() < nsl * S:
                slots = torch.empty(max(nsl, 1) * S * 2, dtype=torch.uint8, device=dev)
                out = torch.empty_like(slots)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if mode == "collector":
                col.run_many(encs, slots, S, cook=ctx, seed=f, out=out)
            else:
                base = 0
                for ci in range(ncon):
                    p = plans[ci]
                    sv = slots[base * S:(base + max(p.n_slots, 1)) * S]
                    ov = out[base * S:(base + max(p.n_slots, 1)) * S]
                    encs[ci].run_cooked(sv, S, ctx, f, out=ov)
                    base += p.n_slots
            e1.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if f >= 2:  # the first flushes pay allocations and run-time compiles
                gpu_ms.append(e0.elapsed_time(e1))
                wall_ms.append((t1 - t0) * 1e3)
                plan_ms.append((t_plan - t0) * 1e3)
                npk_tot += npk
                nev_tot += sum(len(l) for l in lens)
            del inbuf
        for e in encs:
            e.close()
        if col is not None:
            col.close()
        res[mode] = {"run_ms_per_flush": round(statistics.median(gpu_ms), 4),
                     "flush_wall_ms": round(statistics.median(wall_ms), 3),
                     "plan_ms": round(statistics.median(plan_ms), 3),
                     "cooked_packets_per_s_run": round(npk_tot / (sum(gpu_ms) * 1e-3), 1),
                     "packets_per_flush": round(npk_tot / len(gpu_ms), 1)}
    ctx.close()
    res["what"] = ("200 connections x 64-256 datagrams (64-1200 B) per 8 ms flush, -f 20:10 mode 0: "
                   "framing + encode + do_cook into device memory, one collector launch set vs 200 "
                   "rsmi_fenc_run_cooked_dev calls; run = GPU time from the first launch to the last")
    res["speedup_run"] = round(res["per_connection"]["run_ms_per_flush"] /
                               res["collector"]["run_ms_per_flush"], 2)
    return res


def dropin_latency(u, calls=300):
    """Wall time of one level-1 drop-in call (the reference-mangled
    rs_encode2 / rs_decode2 on host buffers, lib/rs.cpp:56-64): RS(20,10),
    1250 B, 5 erasures; median over ``calls`` calls, microseconds."""
    import ctypes as C
    import numpy as np
    n = K + M
    rows = np.random.default_rng(3).integers(0, 256, (n, LEN), dtype=np.uint8)
    arr = (C.c_void_p * n)(*[rows[j].ctypes.data for j in range(n)])
    enc = u.lib().compat["rs_encode2"]
    dec = u.lib().compat["rs_decode2"]
    te = []
    for i in range(calls + 20):
        t0 = time.perf_counter()
        enc(K, n, arr, LEN)
        te.append(time.perf_counter() - t0)
    td = []
    erased = [1, 4, 9, 22, 27]
    for i in range(calls + 20):
        ptrs = (C.c_void_p * n)(*[None if j in erased else rows[j].ctypes.data
                                  for j in range(n)])
        t0 = time.perf_counter()
        rc = dec(K, n, ptrs, LEN)
        td.append(time.perf_counter() - t0)
        if rc:
            raise SystemExit("dropin_latency: rs_decode2 failed")
    # the same calls timed in C (rsmi_dropin_latency), the harness of the
    # reference's per-call figure (cpu_baseline.single_thread): no ctypes
    # dispatch or interpreter time in the number
    L = u.lib()
    pres = np.ones(n, np.uint8)
    pres[erased] = 0
    ce, cd = C.c_double(), C.c_double()
    if L.rsmi_dropin_latency(0, K, n, LEN, None, calls, C.byref(ce)) or \
            L.rsmi_dropin_latency(1, K, n, LEN, pres.ctypes.data, calls, C.byref(cd)):
        raise SystemExit("dropin_latency: rsmi_dropin_latency failed")
    return {"rs_encode2": round(ce.value, 1), "rs_decode2": round(cd.value, 1),
            "calls": calls, "what": "one RS(20,10) 1250-B group per call, host buffers, "
                                    "synchronous; median, timed in C like the reference's per-call figure",
            "python_ctypes": {"rs_encode2": round(statistics.median(te[20:]) * 1e6, 1),
                              "rs_decode2": round(statistics.median(td[20:]) * 1e6, 1),
                              "what": "the same calls from Python through ctypes"}}


def dropin_latency_both(u):
    """The drop-in per-call latency through the default path -- the group
    posted to the resident one-group server (RSMI_OPT_ONE_SERVER: 16
    workgroups polling a doorbell in pinned host memory, no launch per call),
    which reads the pinned staging over PCIe and raises per-workgroup flags --
    and, beside it, the same kernel launched per call and the staged copy
    path (H2D, kernel, D2H, stream sync)."""
    L = u.lib()
    prev = L.rsmi_option(3, 1)
    prev_srv = L.rsmi_option(5, 20000)
    try:
        one = dropin_latency(u)
        L.rsmi_option(5, 0)
        launched = dropin_latency(u)
        L.rsmi_option(3, 0)
        staged = dropin_latency(u)
    finally:
        L.rsmi_option(3, prev)
        L.rsmi_option(5, prev_srv)
    one["what"] += (": posted to the resident server (oneshot.hip k_one_server), which reads pinned staging "
                    "over PCIe; per-workgroup flags polled")
    one["launch_per_call"] = {"rs_encode2": launched["rs_encode2"], "rs_decode2": launched["rs_decode2"],
                              "what": "the same multi-workgroup kernel launched per call (k_one_multi)"}
    one["staged_copy_path"] = {"rs_encode2": staged["rs_encode2"], "rs_decode2": staged["rs_decode2"],
                               "what": "pinned staging, H2D, kernel, D2H, stream sync"}
    return one


def cpu_baseline(buf, present, G, threads):
    """Time the reference codec (oracle/_ref/libref_rs.so: lib/fec.cpp +
    lib/rs.cpp unmodified) on this host -- or the C restatement if the
    reference build is absent -- on the same C1+C2 groups: 1 thread on a
    4,096-group sample and ``threads`` threads on a 65,536-group sample,
    median of 5 reps each, checked against the GPU's parity.  ``value`` is the
    multi-threaded rate; the 1-thread run also gives the reference's per-call
    latency (one rs_encode2 / rs_decode2 per group, lib/rs.cpp:56-64)."""
    import numpy as np
    import platform
    from oracle.cpu import Oracle, Reference

    n = K + M
    host = buf[:min(G, 65536)].cpu().numpy()  # data + GPU parity (+ decoded rows == data)
    pres = present[:min(G, 65536)].cpu().numpy()
    ref = Reference.available()
    lib = Reference() if ref else Oracle()
    kind = "reference" if ref else "port"

    def run(sample, nthreads, reps=5):
        pristine = np.ascontiguousarray(host[:sample])
        gpu_par = pristine[:, K:, :LEN].copy()
        te, td = [], []
        for r in range(reps):
            b = pristine.copy()
            b[:, K:] = 0
            t0 = time.perf_counter()
            if ref:
                lib.encode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample, nthreads)
            else:
                lib.encode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample)
            t1 = time.perf_counter()
            if r == 0 and not (b[:, K:, :LEN] == gpu_par).all():
                raise SystemExit("cpu_baseline: CPU parity differs from GPU parity")
            t2 = time.perf_counter()
            if ref:
                lib.decode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample,
                                 pres[:sample], False, nthreads)
            else:
                lib.decode_batch(K, n, b.reshape(-1), n * STRIDE, STRIDE, LEN, sample,
                                 pres[:sample])
            t3 = time.perf_counter()
            te.append(t1 - t0)
            td.append(t3 - t2)
        tot = [a + b for a, b in zip(te, td)]
        return (2.0 * sample * K * LEN / statistics.median(tot) / 2**30,
                statistics.median(te) / sample, statistics.median(td) / sample)

    one_sample = min(4096, host.shape[0])
    gib1, enc1, dec1 = run(one_sample, 1)
    # the box's CPU share: the CPUs this process may run on, bounded by its
    # cgroup's CPU quota (a 16-CPU quota over 256 affine CPUs throttles 256
    # threads to 16 CPUs' time, and their contention then costs more than it
    # gains -- both runs are reported)
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:  # cgroup v2: "max 100000" or "<quota> <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    share = min(affinity, max(1, int(quota + 0.5))) if quota else affinity
    nthreads = (threads or share) if ref else 1
    many_sample = host.shape[0]
    gibn, _, _ = run(many_sample, nthreads) if nthreads > 1 else (gib1, enc1, dec1)
    side = {}
    for t in sorted({16, affinity} - {nthreads}):
        if ref:
            side[t] = run(many_sample, t, reps=3)[0]
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                 if l.startswith("model name")][0]
    except (OSError, IndexError):
        model = platform.processor()
    return {"value": round(gibn, 3), "unit": "GiB/s", "cores": nthreads, "kind": kind,
            "sample": f"{many_sample} groups RS(20,10)x1250B encode + decode (5 erasures), "
                      f"median of 5 reps, {nthreads} threads (= the box's CPU share: "
                      f"min(sched_getaffinity, cgroup quota)) on {model}",
            "cpu_model": model, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "os_cpu_count": os.cpu_count(),
            "other_thread_counts": {str(t): {"value": round(v, 3), "unit": "GiB/s", "reps": 3}
                                    for t, v in side.items()},
            "single_thread": {"value": round(gib1, 3), "unit": "GiB/s", "cores": 1,
                              "sample": f"{one_sample} groups, median of 5 reps",
                              "rs_encode2_us_per_call": round(enc1 * 1e6, 1),
                              "rs_decode2_us_per_call": round(dec1 * 1e6, 1)}}


if __name__ == "__main__":
    main()
