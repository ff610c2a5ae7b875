"""Decode timing under different launch patterns (C1 encode + C2 decode, RS(20,10)):
back-to-back steps as bench.py runs them, synchronised steps as ab_encode.py
runs them, decode-only back-to-back, and the C2 worst case (5 data erasures
per group) decode-only, and encode-only.  Prints per-pattern mean / median ms."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import udpspeeder_amd as u
from udpspeeder_amd import synth

k, n, ln, G = 20, 30, 1250, 65536
t = torch.empty((G, n, 1280), dtype=torch.uint8, device="cuda")
u.fill_data(t, k, ln, 5)
pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, 0, G, n, 5)).cuda()
# C2 worst case as bench.py's other_configs: every group loses 5 data shards
worst = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED + 1, 0, G, n, 5, limit=k)).cuda()
st = torch.empty(G, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()


def run(pattern, steps=30):
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for i in range(steps):
        ev[i][0].record(s)
        if pattern not in ("dec_only", "worst"):
            u.encode(t, k, n, ln, stream=s)
        ev[i][1].record(s)
        if pattern != "enc_only":
            u.decode(t, worst if pattern == "worst" else pres, k, n, ln, status=st, stream=s)
        ev[i][2].record(s)
        if pattern == "sync":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    enc = [a.elapsed_time(b) for a, b, _ in ev[3:]]
    dec = [b.elapsed_time(c) for _, b, c in ev[3:]]
    print(f"{os.path.basename(os.environ.get('RSMI_LIB', 'default')):24s} {pattern:9s} "
          f"encode mean {statistics.mean(enc):.4f} med {statistics.median(enc):.4f}  "
          f"decode mean {statistics.mean(dec):.4f} med {statistics.median(dec):.4f}", flush=True)


for p in (sys.argv[1].split(",") if len(sys.argv) > 1 else
          ("b2b", "sync", "dec_only", "b2b", "worst", "enc_only")):
    run(p)
