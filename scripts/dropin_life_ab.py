"""Drop-in per-call latency (rsmi_dropin_latency, C-timed) with the resident
server's lifetime at 8 ms and 10 s, alternating (profiles/r06/dropin_life_ab.txt)."""
import ctypes as C, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, udpspeeder_amd as u
L = u.lib()
k, n, ln = 20, 30, 1250
pres = np.ones(n, np.uint8); pres[[1, 4, 9, 22, 27]] = 0
for life in (8, 10000, 8, 10000):
    L.rsmi_option(6, life)
    L.rsmi_quiesce()
    d, e = C.c_double(), C.c_double()
    L.rsmi_dropin_latency(1, k, n, ln, pres.ctypes.data, 300, C.byref(d))
    L.rsmi_dropin_latency(0, k, n, ln, None, 300, C.byref(e))
    print(f"life {life} ms: rs_decode2 {d.value:.1f} us, rs_encode2 {e.value:.1f} us", flush=True)
