"""Measurement only: phase times of k_cook per wave step (8 packets), from a
COOK_TRACE=1 build (RSMI_LIB=udpspeeder_amd/ab/librsmi_ctrace.so), on the bench
workload (every packet C1 emits: 1258 B, key on, device IVs).  Phases: 0-1
length, IV draw and repeat; 1-2 the rounds (CRC, obscure, xor, stores); 2-3
crc unshift + tail overlay; 3-4 tail piece + out_len."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd.cook import CookContext  # noqa: E402

npk, plen, stride = 1966080, 1258, 1312
pk = torch.randint(0, 256, (npk, stride), dtype=torch.uint8, device="cuda")
lens = torch.full((npk,), plen, dtype=torch.int32, device="cuda")
olen = torch.empty_like(lens)
ctx = CookContext(b"bench-key", 0)
steps = (npk + 7) // 8
tr = torch.zeros(steps * 8, dtype=torch.int64, device="cuda")
lib = u.lib()
lib.rsmi_debug_cook_trace.argtypes = [C.c_void_p]
assert lib.rsmi_debug_cook_trace(tr.data_ptr()) == 0
for i in range(60):
    ctx.cook(pk, lens, cap=stride, out_len=olen, seed=i)
torch.cuda.synchronize()
t = tr.view(steps, 8).cpu().numpy().astype(np.int64)
ok = t[:, 4] != 0
t = t[ok]
ph = np.diff(t[:, :5], axis=1)
print(f"wave steps traced {len(t)}; rounds {np.unique(t[:, 5])}")
for i, name in enumerate(["setup (len, IV draw, IV repeat)", "rounds (crc, obscure, xor, store)",
                          "unshift + tail overlay", "tail piece + out_len"]):
    print(f"  {name:36s} median {np.median(ph[:, i]):8.0f}  mean {ph[:, i].mean():8.0f} cycles")
print(f"  total per step median {np.median(t[:, 4] - t[:, 0]):.0f}")
