import os, sys
sys.path.insert(0, os.getcwd())
os.environ["RSMI_DEBUG_PINNED"] = "1"
import torch, numpy as np
import udpspeeder_amd as u
from udpspeeder_amd import synth
k, n, ln, S = 20, 30, 1250, 1280
for G in (9000, 30000, 65536):
    h = torch.zeros((G, n, S), dtype=torch.uint8).pin_memory()
    pres = synth.erasure_present(1, 0, G, n, 5)
    st = u.rs.decode_pinned(h, pres, k, n, ln, chunk_groups=4096)
    print(G, h.numel(), "path", u.lib().rsmi_last_decode_pinned_path(), flush=True)
