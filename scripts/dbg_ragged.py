import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import udpspeeder_amd as u
from oracle.cpu import Oracle
o = Oracle()
rng = np.random.default_rng(5)
G = 300
ks = rng.integers(1, 40, G); ns = ks + rng.integers(0, 30, G); ls = rng.integers(0, 3000, G)
groups, total = u.make_groups(ks, ns, ls)
host = rng.integers(0, 256, total, dtype=np.uint8)
base = torch.from_numpy(host).cuda()
u.encode_ragged(base, groups)
out = base.cpu().numpy()
nbad = 0
for i in range(G):
    d = groups[i]
    seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
    o.encode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1)
    got = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
    exp = seg.reshape(d.n, d.shard_stride)
    diff = got[:, :d.len] != exp[:, :d.len]
    if diff.any():
        nbad += 1
        rows = np.where(diff.any(1))[0]
        cols = np.where(diff.any(0))[0]
        if nbad < 12:
            print(i, "k", d.k, "n", d.n, "len", d.len, "ss", d.shard_stride, "off", d.offset, "rows", rows.tolist()[:8], "cols", cols.min(), cols.max(), len(cols))
print("bad groups", nbad)
