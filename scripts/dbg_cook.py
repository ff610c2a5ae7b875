"""Debug aid: run one random cook batch and report the packets/bytes that differ
from the oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.cpu import CookOracle, cook_ivs, cook_payloads  # noqa: E402
from udpspeeder_amd.cook import CookContext  # noqa: E402

key, flags = (sys.argv[1].encode() if len(sys.argv) > 1 else b""), int(sys.argv[2]) if len(sys.argv) > 2 else 0
o = CookOracle()
npk, stride = 777, 3136
rng = np.random.default_rng(flags * 31 + len(key))
lens = rng.integers(0, 3020, npk).astype(np.int32)
lens[:40] = np.arange(40)
lens[40:60] = 1536 + np.arange(-10, 10)
buf = cook_payloads(0xC0DE + flags, 0, npk, lens, stride)
buf[:, -64:] = 0xA5
iv, ivl = cook_ivs(0xC0DE, 0, npk)
ivl[:33] = np.arange(33)
want = buf.copy()
wout = o.cook_batch(want, stride, lens, iv, ivl, key, flags)
ctx = CookContext(key, flags)
dev = torch.device("cuda:0")
t = torch.from_numpy(buf.copy()).to(dev)
out = ctx.cook(t, torch.from_numpy(lens).to(dev), cap=stride - 64, iv=torch.from_numpy(iv).to(dev),
               iv_len=torch.from_numpy(ivl).to(dev)).cpu().numpy()
got = t.cpu().numpy()
bad = np.nonzero((got != want).any(1))[0]
print("out_len mismatches", int((out != wout).sum()), "packets differing", len(bad))
for i in bad[:25]:
    d = np.nonzero(got[i] != want[i])[0]
    print(f"pk {i} len {lens[i]} ivl {ivl[i]} out {wout[i]} diff bytes {len(d)} first {d[:8]} last {d[-4:]}")
