"""A/B of RSMI_OPT_PARITY_COOK on bench.py's f1_f2 workload (one connection's
1200-B datagrams, mode 0, -f 20:10: 65,536 RS(20,10) groups per batch) through
rsmi_fenc_run_cooked_dev into device memory: two encoders fed the same stream,
one with the parity cooked after the encoder (off), one in its epilogue (on),
runs alternating; every batch's cooked packets compared byte for byte
(within each packet's cooked length).  One JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import udpspeeder_amd as u
from udpspeeder_amd._lib import RSMI_OPT_PARITY_COOK
from udpspeeder_amd.cook import CookContext
from udpspeeder_amd.fec import FecEncoder

G = int(os.environ.get("GROUPS", "65536"))
REPS = int(os.environ.get("REPS", "6"))
dev = torch.device("cuda:0")
plen, npk = 1200, G * 20
lens = np.full(npk, plen, np.int32)
offs = np.arange(npk, dtype=np.uint64) * np.uint64(1216)
inbuf = torch.randint(0, 256, (npk * 1216 + 64,), dtype=torch.uint8, device=dev)
ctx = CookContext(b"bench-key")
encs = {False: FecEncoder("20:10", 0, 1250, 200, seq0=1), True: FecEncoder("20:10", 0, 1250, 200, seq0=1)}
bufs = {}
ts = {False: [], True: []}
used = {False: 0, True: 0}
same = True
for i in range(REPS + 1):
    ol, plan = {}, None
    for on in ([False, True] if i % 2 == 0 else [True, False]):
        u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, int(on))
        p = encs[on].plan(lens, offs, inbuf)
        S = FecEncoder.slot_stride_for(int(p.groups["fec_len"].max()))
        if on not in bufs or bufs[on][0].numel() < p.n_slots * S:
            bufs.pop(on, None)
            sl = torch.empty(p.n_slots * S + 64 * S, dtype=torch.uint8, device=dev)
            bufs[on] = (sl, torch.empty_like(sl))
        slots, out = bufs[on]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ol[on] = encs[on].run_cooked(slots, S, ctx, 11 + i, out=out)
        e1.record()
        torch.cuda.synchronize()
        used[on] = encs[on].last_parity_cooked()
        if i:
            ts[on].append(e0.elapsed_time(e1))
        plan = (p, S)
    p, S = plan
    n = len(p.packets)
    a, b = ol[False][:n], ol[True][:n]
    same = same and torch.equal(a, b)
    # every packet's cooked bytes: [slot * S + 120, + out_len)
    per_slot = torch.zeros(p.n_slots, dtype=torch.int64, device=dev)
    per_slot[torch.from_numpy(p.packets["slot"].astype(np.int64)).to(dev)] = a.to(torch.int64)
    pos = torch.arange(S, device=dev)
    for s0 in range(0, p.n_slots, 1 << 18):  # bounded temporaries
        s1 = min(p.n_slots, s0 + (1 << 18))
        valid = (pos[None, :] >= 120) & (pos[None, :] < 120 + per_slot[s0:s1, None])
        x = bufs[False][1][s0 * S:s1 * S].view(s1 - s0, S)
        y = bufs[True][1][s0 * S:s1 * S].view(s1 - s0, S)
        same = same and bool(((x != y) & valid).sum().item() == 0)
line = {"groups": G, "reps": REPS, "run_ms_off": round(statistics.median(ts[False]), 4),
        "run_ms_on": round(statistics.median(ts[True]), 4),
        "all_off": [round(t, 4) for t in ts[False]], "all_on": [round(t, 4) for t in ts[True]],
        "parity_cook_runs_on": used[True], "parity_cook_runs_off": used[False], "cooked_bytes_identical": same}
print(json.dumps(line), flush=True)
