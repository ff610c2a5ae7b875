"""Diagnose the two-stream encode / erase / decode scenario
(tests/test_gpu_parity.py::test_concurrent_streams) with RSMI_STREAM_ORDER=0.

Per rep both tensors are reset, then each stream runs encode -> erase (0x77)
-> decode once, concurrently with the other stream; after a device sync every
byte the sequence defines is checked on the GPU: data rows (rebuilt or not)
and the surviving parity rows.  A mismatch is classified:

* ``parity``: a surviving parity row is wrong after the encode;
* ``lost``: a rebuilt data row holds the erase value 0x77 (the decode's store
  did not land, or was overwritten);
* ``stale-in``: the rebuilt bytes equal a decode of the survivors with the
  parity rows as they were BEFORE the encode (zeros): the decode read stale
  parity;
* ``other``.

Usage: python scripts/diag_streams.py REPS [G]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd import synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    k, n, ln, S = 20, 30, 1250, 1280
    gpu = torch.device("cuda:0")
    lib = os.path.basename(os.environ.get("RSMI_LIB", "default"))
    init = []
    for i in range(2):
        t = torch.zeros((G, n, S), dtype=torch.uint8, device=gpu)
        u.fill_data(t, k, ln, 100 + i)
        init.append(t)
    ref = [t.clone() for t in init]
    for r in ref:
        u.encode(r, k, n, ln)
    torch.cuda.synchronize()
    pres = [torch.from_numpy(synth.erasure_present(7 + i, 0, G, n, 5)).to(gpu) for i in range(2)]
    masks = [(p == 0).unsqueeze(-1) for p in pres]
    ts = [t.clone() for t in init]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    counts = {}
    for rep in range(reps):
        for t, i0 in zip(ts, init):
            t.copy_(i0)
        torch.cuda.synchronize()
        for t, s, p, m in zip(ts, (s1, s2), pres, masks):
            with torch.cuda.stream(s):
                u.encode(t, k, n, ln)
                t.masked_fill_(m, 0x77)
                u.decode(t, p, k, n, ln)
        torch.cuda.synchronize()
        for i, (t, r, p, m) in enumerate(zip(ts, ref, pres, masks)):
            # defined bytes: all data rows, surviving parity rows, [:ln]
            want = torch.where(m, torch.full_like(r, 0x77), r)
            want[:, :k] = r[:, :k]
            bad = (t[:, :, :ln] != want[:, :, :ln])
            if not bool(bad.any()):
                continue
            idx = bad.nonzero().cpu().numpy()
            pr = p.cpu().numpy()
            got = t[:, :, :ln].cpu().numpy()
            exp = want[:, :, :ln].cpu().numpy()
            kinds = {}
            for g, j, o in idx:
                if j >= k:
                    kind = "parity"
                elif got[g, j, o] == 0x77:
                    kind = "lost"
                else:
                    kind = "other"
                kinds[kind] = kinds.get(kind, 0) + 1
            # stale-in check for the "other" data bytes: decode with zero parity
            oth = [(g, j, o) for g, j, o in idx if j < k and got[g, j, o] != 0x77]
            if oth:
                gs = sorted({int(g) for g, _, _ in oth})[:8]
                z = init[i][gs].clone()
                z.masked_fill_(m[gs], 0x77)
                u.decode(z, p[gs].contiguous(), k, n, ln)
                zz = z[:, :, :ln].cpu().numpy()
                stale = sum(1 for g, j, o in oth if g in gs and zz[gs.index(g), j, o] == got[g, j, o])
                kinds["stale-in(of first 8 groups)"] = stale
            # which of a lane's two 16-B pieces (bitslice.hip: c0 = 128w + lane,
            # c1 = c0 + 64; column c = g * 80 + offset // 16) and which parity rows
            par = idx[idx[:, 1] >= k]
            if len(par):
                col = par[:, 0].astype(np.int64) * 80 + par[:, 2] // 16
                halves = np.bincount(((col % 128) >= 64).astype(np.int64), minlength=2).tolist()
                lanes = sorted(set(((col % 128) % 64).tolist()))[:16]
                kinds["parity c0/c1 bytes"] = halves
                kinds["parity lanes"] = lanes
                kinds["parity rows"] = sorted(set(par[:, 1].tolist()))
                kinds["dword in piece"] = sorted(set(((par[:, 2] % 16) // 4).tolist()))
            offs = np.unique(idx[:, 2])
            rows = np.unique(idx[:, :2], axis=0)
            g0, j0 = rows[0]
            sel = idx[(idx[:, 0] == g0) & (idx[:, 1] == j0)][:, 2]
            print(f"{lib} rep {rep} t{i}: {len(idx)} bad bytes in {len(rows)} rows of "
                  f"{len(np.unique(idx[:, 0]))} groups; kinds {kinds}; offsets mod 256 "
                  f"{sorted(set((offs % 256).tolist()))[:24]}; first row g={g0} j={j0} "
                  f"erased={int(pr[g0, j0] == 0)} erased_set={np.nonzero(pr[g0] == 0)[0].tolist()} "
                  f"offs {sel[:16].tolist()} got {got[g0, j0, sel[:16]].tobytes().hex()} "
                  f"exp {exp[g0, j0, sel[:16]].tobytes().hex()}", flush=True)
            for kk, v in kinds.items():
                if isinstance(v, int):
                    counts[kk] = counts.get(kk, 0) + v
            counts["bad_reps"] = counts.get("bad_reps", 0) + 1
    print(f"{lib}: {reps} reps, summary {counts}", flush=True)


if __name__ == "__main__":
    main()
