"""C1: RS(20,10) encode of 1250-B shards, 65,536 groups, device-resident;
HIP-event time per call after a clock-settle phase (bench.py's _time_ms)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd import synth  # noqa: E402

G, K, N, LEN = 65536, 20, 30, 1250
buf = torch.empty((G, N, 1280), dtype=torch.uint8, device="cuda")
u.fill_data(buf, K, LEN, synth.DATA_SEED)


def time_ms(fn, reps=30, settle_ms=300.0):
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps + 1)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev[1:])


ms = time_ms(lambda: u.encode(buf, K, N, LEN))
print(json.dumps({"c1_encode_ms": round(ms, 4), "frac": round(G * 37500 / (ms * 1e-3) / 8e12, 4)}))
