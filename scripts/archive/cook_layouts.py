"""Where k_cook's time goes with the FEC run's packet layout: the same 1.97 M
packets cooked (device-drawn IVs, key on) in place at a fixed 1312-B stride
(the f2 bench), out of place, at the FEC slot layout (1408-B slots, packet at
+120), and with lengths 1211 (the f1_f2 run's packets).  HIP-event median of
10 launches each; one JSON line per layout."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from udpspeeder_amd.cook import CookContext  # noqa: E402

npk = 65536 * 30
ctx = CookContext(b"bench-key")


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


for name, stride, off, ln, oop in [("f2_inplace_1312", 1312, 0, 1258, False),
                                   ("f2_outofplace_1312", 1312, 0, 1258, True),
                                   ("slot_inplace_1408_off120", 1408, 120, 1211, False),
                                   ("slot_outofplace_1408_off120", 1408, 120, 1211, True),
                                   ("len1211_inplace_1312", 1312, 0, 1211, False)]:
    buf = torch.randint(0, 256, (npk * stride + 256,), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(buf) if oop else None
    lens = torch.full((npk,), ln, dtype=torch.int32, device="cuda")
    offs = torch.arange(npk, dtype=torch.int64, device="cuda") * stride + off
    cap = stride - off
    if oop:
        f = lambda: ctx.cook_to(buf, lens, out, cap=cap, offsets=offs, seed=3)
    else:
        f = lambda: ctx.cook(buf, lens, cap=cap, offsets=offs, seed=3)
    t = timed(f)
    print(json.dumps({"layout": name, "ms": round(t, 4), "Mpps": round(npk / t / 1e3, 1)}), flush=True)
    del buf, out
    torch.cuda.empty_cache()
