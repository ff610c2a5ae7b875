import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import udpspeeder_amd as u
from oracle.cpu import Oracle
o = Oracle()
for (k, n, ln, G) in [(20, 30, 1250, 4), (20, 30, 32, 1), (1, 4, 64, 3), (20, 30, 1250, 300)]:
    S = (ln + 15) // 16 * 16
    rng = np.random.default_rng(1)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    t = torch.from_numpy(buf).cuda()
    u.encode(t, k, n, ln)
    torch.cuda.synchronize()
    out = t.cpu().numpy()
    o.encode_batch(k, n, buf.reshape(-1), n * S, S, ln, G)
    d = out[:, :, :ln] != buf[:, :, :ln]
    print((k, n, ln, G), "mismatch bytes", int(d.sum()), "rows", sorted(set(np.where(d)[1].tolist()))[:12])
    if d.any():
        g, r, c = [x[0] for x in np.where(d)]
        print("  first", g, r, c, "got", out[g, r, c:c+8].tolist(), "exp", buf[g, r, c:c+8].tolist())
        # bit pattern diff at first 32 bytes of row
        print("  xor", (out[0, r, :32] ^ buf[0, r, :32]).tolist())
