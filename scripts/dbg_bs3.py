import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import udpspeeder_amd as u
from oracle.cpu import Reference
o = Reference()
k, n, ln, G, S = 20, 30, 1250, 65536, 1280
t = torch.zeros((G, n, S), dtype=torch.uint8, device="cuda")
u.fill_data(t, k, ln, 77)
torch.cuda.synchronize()
buf = t.cpu().numpy()
ref = buf.copy()
o.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G, 16)
for rep in range(3):
    t[:, k:] = 0
    u.encode(t, k, n, ln)
    torch.cuda.synchronize()
    out = t.cpu().numpy()
    d = out[:, :, :ln] != ref[:, :, :ln]
    bg = np.where(d.any(axis=(1, 2)))[0]
    print(os.environ.get("RSMI_LIB", "default"), "rep", rep, "bad groups", len(bg), flush=True)
