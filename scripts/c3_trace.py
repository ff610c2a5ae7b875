"""Measurement only: per-group phase times of the C3 class decode kernels, from a
DEC_TRACE=1 build (RSMI_LIB=udpspeeder_amd/ab/librsmi_trace.so).  Each decoded
group records s_memtime at its start, after survivor selection, after the
Gauss-Jordan (+ coefficient expansion) and after its survivor stream; each wave
records its kernel entry and the time its tables were ready.  Prints, per tile
width class, the mean phase times in cycles and how long waves live."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd import synth  # noqa: E402

G = 65536
table = u.rs_from_str(synth.C3_FEC)
ks, ms, ls = synth.ragged_mix(synth.RAGGED_SEED, 0, G, [y for _, y in table])
groups, total = u.make_groups(ks, ks + ms, ls)
base = torch.zeros(total, dtype=torch.uint8, device="cuda")
dg = u.rs.groups_to_device(groups)
u.rs.fill_ragged(base, dg, G, synth.DATA_SEED)
plan = u.rs.RaggedPlan(groups)
plan.encode(base)
flags = synth.ragged_erasures(synth.ERASE_SEED, 0, ks + ms, ms, 5)
bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to("cuda")
st = torch.empty(G, dtype=torch.int32, device="cuda")
tr = torch.zeros(G * 8, dtype=torch.int64, device="cuda")
lib = u.lib()
lib.rsmi_debug_dec_trace.argtypes = [C.c_void_p]
assert lib.rsmi_debug_dec_trace(tr.data_ptr()) == 0
for _ in range(200):  # settle the clocks; the last call's stamps stay
    plan.decode(base, bits, status=st)
torch.cuda.synchronize()
assert int((st != 0).sum()) == 0
t = tr.view(G, 8).cpu().numpy().astype(np.int64)
ok = t[:, 4] != 0
info = t[:, 4]
W = info & 0xFF
k = (info >> 8) & 0xFF
e = (info >> 16) & 0xFF
ln = info >> 32
print(f"traced groups {int(ok.sum())} of {G}")
for w in (5, 4, 2, 1):
    m = ok & (W == w)
    if not m.any():
        continue
    sel = t[m, 1] - t[m, 0]
    gj = t[m, 2] - t[m, 1]
    run = t[m, 3] - t[m, 2]
    tot = t[m, 3] - t[m, 0]
    waves = np.unique(t[m, 5])
    # per wave: entry -> tables ready, and entry -> last group end
    wv = t[m, 5]
    order = np.argsort(wv, kind="stable")
    wv_s, t3_s, t0_s = wv[order], t[m, 3][order], t[m, 0][order]
    starts = np.r_[0, np.flatnonzero(np.diff(wv_s)) + 1]
    last_end = np.maximum.reduceat(t3_s, starts)
    first_start = np.minimum.reduceat(t0_s, starts)
    tk0 = t[m, 6][order][starts]
    tk1 = t[m, 7][order][starts]
    ngw = np.diff(np.r_[starts, len(wv_s)])
    print(f"W={w}: groups {int(m.sum())}, waves {len(waves)} ({ngw.mean():.2f} groups/wave), "
          f"k mean {k[m].mean():.1f}, e mean {e[m].mean():.2f}, len mean {ln[m].mean():.0f}")
    print(f"   per group cycles: select {np.median(sel):.0f} (mean {sel.mean():.0f}), "
          f"gauss-jordan+expand {np.median(gj):.0f} (mean {gj.mean():.0f}), "
          f"stream {np.median(run):.0f} (mean {run.mean():.0f}), total {np.median(tot):.0f} (mean {tot.mean():.0f})")
    print(f"   per wave cycles: entry->tables {np.median(tk1 - tk0):.0f}, tables->first group "
          f"{np.median(first_start - tk1):.0f}, entry->last end {np.median(last_end - tk0):.0f} "
          f"(p90 {np.percentile(last_end - tk0, 90):.0f}, max {np.max(last_end - tk0):.0f})")
    for kk in (2, 6, 12, 20):
        mk = m & (k >= kk - 2) & (k <= kk)
        if mk.any():
            print(f"   k in [{kk - 2},{kk}]: gj {np.median(t[mk, 2] - t[mk, 1]):.0f}, "
                  f"stream {np.median(t[mk, 3] - t[mk, 2]):.0f}, n {int(mk.sum())}")
