"""Do the framing run and the cook kernel share the GPU productively?  Times
(HIP events, median of 7) one batch's rsmi_fenc_run_dev (k_frame + encode) and
an independent k_cook over 1.31 M packets of 1211 B, alone and launched
together on two streams."""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from udpspeeder_amd.cook import CookContext  # noqa: E402
from udpspeeder_amd.fec import FecEncoder  # noqa: E402

groups = 65536
npk = groups * 20
lens = np.full(npk, 1200, np.int32)
offs = np.arange(npk, dtype=np.uint64) * np.uint64(1216)
inbuf = torch.randint(0, 256, (npk * 1216 + 64,), dtype=torch.uint8, device="cuda")
enc = FecEncoder("20:10", 0, 1250, 200, seq0=1)
ctx = CookContext(b"bench-key")
ncook = npk
cbuf = torch.randint(0, 256, (ncook * 1408 + 256,), dtype=torch.uint8, device="cuda")
cout = torch.empty_like(cbuf)
clen = torch.full((ncook,), 1211, dtype=torch.int32, device="cuda")
coff = torch.arange(ncook, dtype=torch.int64, device="cuda") * 1408 + 120
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
slots = None


def plan():
    global slots
    p = enc.plan(lens, offs, inbuf)
    S = FecEncoder.slot_stride_for(int(p.groups["fec_len"].max()))
    if slots is None or slots.numel() < p.n_slots * S:
        slots = torch.empty(p.n_slots * S + 64 * S, dtype=torch.uint8, device="cuda")
    return S


def run(frame, cook):
    S = plan() if frame else 0
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s1)
    s2.wait_event(a)
    if frame:
        enc.run(slots, S, stream=s1)
    if cook:
        ctx.cook_to(cbuf, clen, cout, cap=1288, offsets=coff, seed=3, stream=s2)
    e2 = torch.cuda.Event()
    e2.record(s2)
    s1.wait_event(e2)
    b.record(s1)
    torch.cuda.synchronize()
    return a.elapsed_time(b)


for name, f, c in [("frame_encode", 1, 0), ("cook", 0, 1), ("both", 1, 1)]:
    ts = [run(f, c) for _ in range(9)][2:]
    print(json.dumps({"what": name, "ms": round(statistics.median(ts), 4)}), flush=True)
