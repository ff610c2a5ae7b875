"""Debug: GPU framing vs the restatement, per packet, for the golden cases."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.fec_frame import EncodeManager
from oracle.gen_golden_fec import CASES, case_events
from tests.test_fec_frame import _run_gpu
from udpspeeder_amd.fec import FecEncoder

for ci, (name, rs, mode, mtu, ql, n, lmax, fpm, zpm) in enumerate(CASES):
    if mode: continue
    lens, ev = case_events(ci, n, lmax, fpm, zpm)
    enc = FecEncoder(rs, mode, mtu, ql, seq0=5)
    em = EncodeManager(rs, mode, mtu, ql, 5)
    exp = []
    for i, e in enumerate(ev):
        em.input(e)
        exp += [(p, i) for p in em.output()]
    out = _run_gpu(enc, lens, ev, np.array([0, n]), torch)
    bad = [i for i, (a, b) in enumerate(zip(out, exp)) if a != b and a[0][7] < a[0][5]]
    print(name, len(out), len(exp), "bad data pk", len(bad))
    # group blob structure for the first bad data packet
    for i in bad[:4]:
        a, b = out[i][0], exp[i][0]
        k, idx = a[5], a[7]
        g0 = i - idx
        fec_len = len(a) - 8
        blob = b"".join(exp[g0 + j][0][8:] for j in range(k))
        cnt = int.from_bytes(blob[:4], "big"); pos = 4; offs = []
        for _ in range(cnt):
            offs.append(pos); pos += 2 + int.from_bytes(blob[pos:pos + 2], "big")
        for d in [j for j in range(8, len(a)) if a[j] != b[j]][:3]:
            bp = idx * fec_len + d - 8
            near = [o for o in offs if abs(o - bp) < 24]
            print(f"  pk{i} idx{idx} byte{d} blobpos {bp} piece_off {(d-8)%16} got {a[d]:02x} exp {b[d]:02x}",
                  "records near", [(o, o - bp) for o in near], "blob_len", pos)
