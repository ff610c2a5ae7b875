"""Per-call latency of the level-1 drop-in's rs_decode2 (RS(20,10), 1250 B, 5
erasures) through the resident server, the per-call launch and the staged
path."""
import ctypes as C
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import udpspeeder_amd as u  # noqa: E402

L = u.lib()
k, n, ln = 20, 30, 1250
rows = np.random.default_rng(3).integers(0, 256, (n, ln), dtype=np.uint8)
dec, enc = L.compat["rs_decode2"], L.compat["rs_encode2"]
erased = {1, 4, 9, 22, 27}
arr = (C.c_void_p * n)(*[rows[j].ctypes.data for j in range(n)])


def med(calls=400):
    td, te = [], []
    for i in range(calls + 20):
        ptrs = (C.c_void_p * n)(*[None if j in erased else rows[j].ctypes.data for j in range(n)])
        t0 = time.perf_counter()
        assert dec(k, n, ptrs, ln) == 0
        td.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        enc(k, n, arr, ln)
        te.append(time.perf_counter() - t0)
    out = {"rs_decode2_us": round(statistics.median(td[20:]) * 1e6, 2),
           "rs_encode2_us": round(statistics.median(te[20:]) * 1e6, 2)}
    pres = np.ones(n, np.uint8)
    pres[list(erased)] = 0
    cd, ce = C.c_double(), C.c_double()
    assert L.rsmi_dropin_latency(1, k, n, ln, pres.ctypes.data, calls, C.byref(cd)) == 0
    assert L.rsmi_dropin_latency(0, k, n, ln, None, calls, C.byref(ce)) == 0
    out["c_timed"] = {"rs_decode2_us": round(cd.value, 2), "rs_encode2_us": round(ce.value, 2)}
    return out


res = {}
L.rsmi_option(3, 1)
L.rsmi_option(5, 20000)
res["server"] = med()
L.rsmi_option(5, 0)
res["launch_per_call"] = med()
L.rsmi_option(3, 0)
res["staged"] = med()
L.rsmi_option(3, 1)
print(json.dumps(res))
