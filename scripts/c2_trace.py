"""Measurement only: per-group phase times of the uniform fused decode
(k_decode_fused) on C2, from a DEC_TRACE=1 build (RSMI_LIB=udpspeeder_amd/ab/
librsmi_trace.so).  Each decoded group records s_memtime at its start, after
survivor selection, after the elimination + coefficient expansion and after
its survivor stream.  Prints the median phase cycles per erasure count e."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd import synth  # noqa: E402

G, K, N, LEN = 65536, 20, 30, 1250
buf = torch.empty((G, N, 1280), dtype=torch.uint8, device="cuda")
u.fill_data(buf, K, LEN, synth.DATA_SEED)
u.encode(buf, K, N, LEN)
for name, lim in (("C2 random 5-of-30", 0), ("C2 worst: 5 data erasures", K)):
    pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, 0, G, N, 5, limit=lim)).to("cuda")
    st = torch.empty(G, dtype=torch.int32, device="cuda")
    tr = torch.zeros(G * 8, dtype=torch.int64, device="cuda")
    lib = u.lib()
    lib.rsmi_debug_dec_trace.argtypes = [C.c_void_p]
    assert lib.rsmi_debug_dec_trace(tr.data_ptr()) == 0
    for _ in range(300):  # settle the clocks; the last call's stamps stay
        u.decode(buf, pres, K, N, LEN, status=st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    t = tr.view(G, 8).cpu().numpy().astype(np.int64)
    ok = t[:, 4] != 0
    e = (t[:, 4] >> 16) & 0xFF
    print(f"{name}: traced groups {int(ok.sum())} of {G}")
    sel, gj, run, tot = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 3] - t[:, 0]
    for ee in range(1, 6):
        m = ok & (e == ee)
        if m.any():
            print(f"  e={ee}: n {int(m.sum()):6d}  select {np.median(sel[m]):7.0f}  elim+expand "
                  f"{np.median(gj[m]):7.0f}  stream {np.median(run[m]):8.0f}  total {np.median(tot[m]):8.0f}")
    m = ok
    print(f"  all : select {sel[m].mean():7.0f}  elim+expand {gj[m].mean():7.0f}  stream "
          f"{run[m].mean():8.0f}  total {tot[m].mean():8.0f} (means)")
    lib.rsmi_debug_dec_trace(None)
