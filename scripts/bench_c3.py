"""C3: ragged mode-0 mix RS encode -- k~U{1..20}, m from -f 1:3,2:4,10:6,20:10,
len~U[64..1250], 65536 groups; device-resident; kernel time via HIP events."""
import os, sys, statistics, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import udpspeeder_amd as u
from udpspeeder_amd import synth
G = 65536
table = u.rs_from_str(synth.C3_FEC)
ks, ms, ls = synth.ragged_mix(synth.RAGGED_SEED, 0, G, [y for _, y in table])
groups, total = u.make_groups(ks, ks + ms, ls, align=int(os.environ.get("ALIGN", "16")))
base = torch.zeros(total, dtype=torch.uint8, device="cuda")
dg = u.rs.groups_to_device(groups)
u.rs.fill_ragged(base, dg, G, synth.DATA_SEED)
for kk in set(zip(ks.tolist(), (ks + ms).tolist())):
    u.prepare_code(*kk)
plan = u.rs.RaggedPlan(groups)


def time_ms(fn, reps=20, settle_ms=150.0):
    """median per-call time, calls back to back after a clock-settle phase
    (bench.py's _time_ms)"""
    import time
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


t = time_ms(lambda: plan.encode(base))
alg = int(((ks + ms) * ls).sum())
print(json.dumps({"bitslice_plan": plan.bitslice, "c3_encode_ms": t, "payload_GiBps": float((ks * ls).sum()) / (t * 1e-3) / 2**30,
                  "alg_GBps": alg / (t * 1e-3) / 1e9, "alg_bytes": alg, "buffer_bytes": total}))
# C3 decode: min(5, m) random erasures per group on the encoded batch (bench.py's c3 line)
flags = synth.ragged_erasures(synth.ERASE_SEED, 0, ks + ms, ms, 5)
bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to("cuda")
st = torch.empty(G, dtype=torch.int32, device="cuda")
clean = base.clone()
# rebuilt rows equal the erased ones, so repeated decodes leave the batch unchanged
td = time_ms(lambda: plan.decode(base, bits, status=st))
assert int((st != 0).sum()) == 0 and torch.equal(base, clean)
e = ((flags[:, :20] == 0) & (np.arange(20)[None, :] < ks[:, None])).sum(1)
dalg = int(((ks + e) * ls).sum())
print(json.dumps({"c3_decode_ms": td, "alg_GBps": dalg / (td * 1e-3) / 1e9, "frac": dalg / (td * 1e-3) / 8e12}))
# the reference's placement (rebuilt rows over the parity survivors): the parity
# slots change, so each timed call decodes a different input -- same work
sm = torch.empty((G, 20), dtype=torch.uint8, device="cuda")
tr = time_ms(lambda: plan.decode(base, bits, status=st, placement="reference", slot_map=sm))
base.copy_(clean)
print(json.dumps({"c3_decode_ref_ms": tr, "frac": dalg / (tr * 1e-3) / 8e12}))
