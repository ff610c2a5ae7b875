"""C2: RS(20,10) decode of 1250-B shards, 65,536 groups, 5 random erasures per
group (and the worst case, 5 data erasures); device-resident, HIP-event time
per call after a clock-settle phase (bench.py's _time_ms)."""
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
u.encode(buf, K, N, LEN)


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


out = {}
smap = torch.empty((G, K), dtype=torch.uint8, device="cuda")
for name, lim in (("c2_random", 0), ("c2_worst", K)):
    pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED + (1 if lim else 0), 0, G, N, 5,
                                                  limit=lim)).to("cuda")
    st = torch.empty(G, dtype=torch.int32, device="cuda")
    e = (pres[:, :K] == 0).sum(1).cpu()
    alg = int(((e > 0) * K * LEN).sum() + (e * LEN).sum())
    for place in ("own", "ref"):
        if place == "own":
            ms = time_ms(lambda: u.decode(buf, pres, K, N, LEN, status=st))
        else:  # the reference's placement (over the parity survivors; the bytes read change, not the work)
            ms = time_ms(lambda: u.decode(buf, pres, K, N, LEN, status=st, placement="reference", slot_map=smap))
            u.encode(buf, K, N, LEN)
        assert int((st != 0).sum()) == 0
        out[f"{name}_{place}"] = {"decode_ms": round(ms, 4), "frac": round(alg / (ms * 1e-3) / 8e12, 4)}
print(json.dumps(out))
