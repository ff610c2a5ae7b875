"""A/B timing of the RS(20,10) C1 encode and C2 decode (bench.py's step; PLACE=reference for the
reference placement) for the library named by RSMI_LIB."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import udpspeeder_amd as u
from udpspeeder_amd import synth
k, n, ln, G = 20, 30, 1250, 65536
PLACE = os.environ.get("PLACE", "own")  # the decode's placement (bench.py's step: own slots)
t = torch.empty((G, n, 1280), dtype=torch.uint8, device="cuda")
u.fill_data(t, k, ln, 5)
pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, 0, G, n, 5)).cuda()
st = torch.empty(G, dtype=torch.int32, device="cuda")
sm = torch.empty((G, k), dtype=torch.uint8, device="cuda")
enc, dec = [], []
for i in range(40):
    a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    a.record(); u.encode(t, k, n, ln); b.record()
    if PLACE == "own":
        u.decode(t, pres, k, n, ln, status=st)
    else:
        u.decode(t, pres, k, n, ln, status=st, placement="reference", slot_map=sm)
    c.record()
    torch.cuda.synchronize()
    if i >= 5:
        enc.append(a.elapsed_time(b)); dec.append(b.elapsed_time(c))
me, md = statistics.median(enc), statistics.median(dec)
print(f"{os.path.basename(os.environ.get('RSMI_LIB', 'default'))} {PLACE}: encode {me:.4f} ms "
      f"({G * 37500 / me / 1e6:.0f} GB/s alg)  decode {md:.4f} ms  bad={int((st != 0).sum())}", flush=True)
