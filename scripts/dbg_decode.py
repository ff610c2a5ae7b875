import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import udpspeeder_amd as u
from oracle.cpu import Oracle
o = Oracle()
k, n, ln, ner = 20, 30, 1250, 5
G = 41; S = 1264
rng = np.random.default_rng(k + n + ln)
buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
present = np.ones((G, n), np.uint8)
for g in range(G):
    e = rng.integers(0, ner + 2)
    present[g, rng.choice(n, min(e, n), replace=False)] = 0
ref = buf.copy()
st_ref = o.decode_batch(k, n, ref.reshape(-1), n * S, S, ln, G, present)
t = torch.from_numpy(buf).cuda()
st = u.decode(t, torch.from_numpy(present).cuda(), k, n, ln).cpu().numpy()
out = t.cpu().numpy()
print("status eq", (st == st_ref).all())
for g in range(G):
    bad = [(j, int(np.argmax(out[g, j, :ln] != ref[g, j, :ln])), int((out[g, j, :ln] != ref[g, j, :ln]).sum())) for j in range(n) if not (out[g, j, :ln] == ref[g, j, :ln]).all()]
    if bad:
        print("group", g, "erased", np.where(present[g] == 0)[0].tolist(), "bad rows (row, first, count)", bad)
