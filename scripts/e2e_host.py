"""End-to-end (host memory -> GPU -> host memory) RS(20,10) encode rate.

Pinned host buffers hold the 65536 groups' data shards [G][k][1280] and receive
parity [G][m][1280]; librsmi's rsmi_encode_pinned pipelines chunks
H2D -> bit-sliced encode -> D2H on three streams.  Also reports the raw pinned
H2D / D2H copy rates for the same byte counts (the PCIe ceiling)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import udpspeeder_amd as u
k, n, ln, G, S = 20, 30, 1250, 65536, 1280
m = n - k
dev = torch.device("cuda:0")
# E2E_DEVICES="0,0": the host entry points split over that device list
# (rsmi_use_devices; one worker thread, streams and pipelines per entry)
DEVS = [int(x) for x in os.environ.get("E2E_DEVICES", "").split(",") if x != ""]
if DEVS:
    u.rs.set_devices(DEVS)
data = torch.empty((G, k, S), dtype=torch.uint8).pin_memory()
par = torch.empty((G, m, S), dtype=torch.uint8).pin_memory()
tmp = torch.empty((G, n, S), dtype=torch.uint8, device=dev)
u.fill_data(tmp, k, ln, 11)
data.copy_(tmp[:, :k])
res = {}
for chunk in (2048, 4096, 8192, 16384):
    u.rs.encode_pinned(data, par, k, n, ln, chunk_groups=chunk)  # warm
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        u.rs.encode_pinned(data, par, k, n, ln, chunk_groups=chunk)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    res[f"chunk{chunk}"] = {"s": t, "payload_GiBps": G * k * ln / t / 2**30,
                            "groups_per_s": G / t}
# parity check against the device path
u.encode(tmp, k, n, ln)
assert torch.equal(par[:, :, :ln], tmp[:, k:, :ln].cpu())
# raw copy ceilings for the same bytes
dd = torch.empty((G, k, S), dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter(); dd.copy_(data, non_blocking=True); torch.cuda.synchronize()
h2d = data.numel() / (time.perf_counter() - t0) / 1e9
t0 = time.perf_counter(); data.copy_(dd, non_blocking=True); torch.cuda.synchronize()
d2h = data.numel() / (time.perf_counter() - t0) / 1e9
res["raw_h2d_GBps"] = h2d
res["raw_d2h_GBps"] = d2h
res["devices"] = u.rs.get_devices() or "current"
print(json.dumps(res, indent=1))

# ---- end-to-end decode.  Pinned shards: zero-copy -- the fused decode kernel
# reads only the k survivors it selects from host memory over PCIe and writes
# only the rebuilt rows back.  Pageable shards: the staged pipeline (whole
# groups H2D, decode, data rows D2H).
import numpy as np
from udpspeeder_amd import synth
shards = torch.empty((G, n, S), dtype=torch.uint8).pin_memory()
u.encode(tmp, k, n, ln)
shards.copy_(tmp)
pres = synth.erasure_present(synth.ERASE_SEED, 0, G, n, 5)
shards[torch.from_numpy(pres == 0)] = 0xA5
pageable = shards.numpy().copy()
e_rows = int((pres[:, :k] == 0).sum())
dres = {"survivor_bytes_per_group": k * S, "rebuilt_bytes_per_group": e_rows * S / G}
for name, buf, chunk in (("zero_copy_pinned", shards, 4096), ("staged_pageable", pageable, 4096),
                         ("staged_pageable_8192", pageable, 8192)):
    u.rs.decode_pinned(buf, pres, k, n, ln, chunk_groups=chunk)
    path = u.lib().rsmi_last_decode_pinned_path()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        st = u.rs.decode_pinned(buf, pres, k, n, ln, chunk_groups=chunk)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    assert (st == 0).all()
    dres[name] = {"s": t, "payload_GiBps": G * k * ln / t / 2**30, "groups_per_s": G / t,
                  "path": {1: "zero-copy", 2: "staged"}[path],
                  "pcie_GBps": (G * k * S + e_rows * S) / t / 1e9 if path == 1 else None}
assert torch.equal(shards[:, :k, :ln], tmp[:, :k, :ln].cpu())
assert (pageable[:, :k, :ln] == tmp[:, :k, :ln].cpu().numpy()).all()
print(json.dumps({"decode_e2e": dres}, indent=1))

# ---- end-to-end C3 (the mode-0 mix) through the ragged host entries: each
# chunk's contiguous span H2D, ragged encode / decode, span D2H; with
# E2E_DEVICES the groups split by summed n * len (rsmi_encode_ragged_pinned)
table = u.rs_from_str(synth.C3_FEC)
ks, ms_, ls = synth.ragged_mix(synth.RAGGED_SEED, 0, G, [y for _, y in table])
groups, total = u.make_groups(ks, ks + ms_, ls)
rb = torch.zeros(total, dtype=torch.uint8).pin_memory()
dtmp = torch.zeros(total, dtype=torch.uint8, device=dev)
u.rs.fill_ragged(dtmp, u.rs.groups_to_device(groups, dev), G, synth.DATA_SEED)
rb.copy_(dtmp)
payload = float((ks * ls).sum())
span = float(((ks + ms_) * np.array([g.shard_stride for g in groups])).sum())
flags = synth.ragged_erasures(synth.ERASE_SEED, 0, ks + ms_, ms_, 5)
bits = synth.present_bits(flags)
rres = {"groups": G, "payload_bytes": payload, "span_bytes_each_way": span}
for chunk in (4096, 16384):
    for op in ("encode", "decode"):
        fn = ((lambda: u.rs.encode_ragged_pinned(rb, groups, chunk_groups=chunk)) if op == "encode" else
              (lambda: u.rs.decode_ragged_pinned(rb, groups, bits, chunk_groups=chunk)))
        fn()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        rres[f"{op}_chunk{chunk}"] = {"s": t, "payload_GiBps": payload / t / 2**30,
                                      "pcie_GBps_both_ways": 2 * span / t / 1e9}
# the encode's parity against the device path
plan = u.rs.RaggedPlan(groups)
plan.encode(dtmp)
torch.cuda.synchronize()
plan.close()
hb, db = rb.numpy(), dtmp.cpu().numpy()
for g in range(0, G, 31):  # payload bytes of every row (the pad bytes may differ between encoders)
    d = groups[g]
    rows = lambda x: x[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)[:, :d.len]
    assert (rows(hb) == rows(db)).all(), g
rres["devices"] = u.rs.get_devices() or "current"
print(json.dumps({"c3_ragged_e2e": rres}, indent=1))
