import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import udpspeeder_amd as u
from oracle.cpu import Oracle, Reference
o = Reference() if Reference.available() else Oracle()
k, n, ln = 20, 30, 1250
for G in [4096, 65536]:
    S = 1280
    t = torch.zeros((G, n, S), dtype=torch.uint8, device="cuda")
    u.fill_data(t, k, ln, 77)
    torch.cuda.synchronize()
    buf = t.cpu().numpy()
    for rep in range(2):
        u.encode(t, k, n, ln)
        torch.cuda.synchronize()
        out = t.cpu().numpy()
        ref = buf.copy()
        o.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G, 16) if isinstance(o, Reference) else o.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G)
        d = out[:, :, :ln] != ref[:, :, :ln]
        bg = np.where(d.any(axis=(1, 2)))[0]
        print("G", G, "rep", rep, "bad groups", len(bg), bg[:10].tolist(), flush=True)
        if len(bg):
            g = bg[0]
            rows = np.where(d[g].any(1))[0]; cols = np.where(d[g].any(0))[0]
            print("   g", g, "rows", rows.tolist(), "cols", cols.min(), cols.max(), len(cols))
            print("   bad col histogram (16B pieces):", np.bincount(np.where(d.any(axis=1))[1] // 16, minlength=79)[:79].tolist())
