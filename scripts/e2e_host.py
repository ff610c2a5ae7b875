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
# (rsmi_set_devices; one worker thread, streams and pipelines per entry)
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
