"""Debug: the two-stream encode / erase / decode scenario of
tests/test_gpu_parity.py::test_concurrent_streams, repeated, reporting which
groups and rows come out wrong for the library named by RSMI_LIB."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd import synth  # noqa: E402
from oracle.cpu import Oracle  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    two = (sys.argv[2] != "one") if len(sys.argv) > 2 else True
    # which steps are librsmi's: "both", "enc" (torch restores erased rows from
    # the clean copy) or "dec" (torch writes the parity rows from the clean copy)
    which = sys.argv[3] if len(sys.argv) > 3 else "both"
    k, n, ln, G = 20, 30, 1250, 2048
    gpu = torch.device("cuda:0")
    orc = Oracle()
    lib = os.path.basename(os.environ.get("RSMI_LIB", "default"))
    if os.environ.get("DBG_NOFUSED"):  # the two-kernel decode instead of the fused one
        from udpspeeder_amd import rs as _rs
        _rs.set_fused_decode(False)
        lib += "/nofused"
    for rep in range(reps):
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        if not two:
            s2 = s1
        ts = [torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu) for _ in range(2)]
        for i, t in enumerate(ts):
            u.fill_data(t, k, ln, 100 + i)
        torch.cuda.synchronize()
        ref = [t.cpu().numpy() for t in ts]
        for r in ref:
            orc.encode_batch(k, n, r.reshape(-1), n * 1280, 1280, ln, G)
        clean = [torch.from_numpy(r).to(gpu) for r in ref]
        pres = [torch.from_numpy(synth.erasure_present(7 + i, 0, G, n, 5)).to(gpu) for i in range(2)]
        noise = torch.ones(64 << 20, dtype=torch.int32, device=gpu) if which == "noise" else None
        torch.cuda.synchronize()
        for _ in range(3):
            for ti, (t, s, p, c) in enumerate(zip(ts, (s1, s2), pres, clean)):
                if which == "noise" and ti == 1:  # stream 2 runs torch work only
                    with torch.cuda.stream(s):
                        for _ in range(4):
                            noise.mul_(3).add_(1)
                    continue
                with torch.cuda.stream(s):
                    if which == "dec":  # ("noise": both steps are librsmi's on stream 1)
                        t[:, k:, :ln] = c[:, k:, :ln]
                    else:
                        u.encode(t, k, n, ln)
                    m = (p == 0).unsqueeze(-1)
                    if not os.environ.get("DBG_NOFILL"):  # erased rows keep their bytes
                        t.masked_fill_(m, 0x77)
                    if which == "enc":
                        t[:, :, :ln] = torch.where(m, c, t)[:, :, :ln]
                    else:
                        u.decode(t, p, k, n, ln)
        torch.cuda.synchronize()
        msg = []
        for i, (t, r) in enumerate(zip(ts, ref)):
            if which == "noise" and i == 1:
                continue
            out = t.cpu().numpy()
            bad = (out[:, :k, :ln] != r[:, :k, :ln])
            rows = np.argwhere(bad.any(axis=2))
            pr = pres[i].cpu().numpy()
            if len(rows):
                g0, j0 = rows[0]
                erased_bad = int(sum(pr[g, j] == 0 for g, j in rows))
                cols = np.nonzero(bad[g0, j0])[0]
                msg.append(f"t{i}: {len(rows)} bad rows in {len(np.unique(rows[:, 0]))} groups "
                           f"({erased_bad} of them rebuilt rows); first g={g0} j={j0} "
                           f"bytes {cols.min()}..{cols.max()} ({len(cols)})")
                if os.environ.get("DBG_DETAIL"):
                    pg = pr[g0]
                    msg.append(f"\n   erased {np.nonzero(pg == 0)[0].tolist()} bad rows of g: "
                               f"{rows[rows[:, 0] == g0][:, 1].tolist()} offsets {cols.tolist()}"
                               f"\n   got {out[g0, j0, cols].tobytes().hex()}"
                               f"\n   exp {r[g0, j0, cols].tobytes().hex()}")
                    # parity rows of that group: are they right (encode) ?
                    pbad = np.argwhere(out[g0, k:, :ln] != r[g0, k:, :ln])
                    msg.append(f"\n   parity diffs in g: {len(pbad)} rows/offs "
                               f"{sorted(set((k + pbad[:, 0]).tolist()))} {sorted(set(pbad[:, 1].tolist()))[:40]}")
        print(f"{lib} {which} rep {rep} {'two' if two else 'one'} stream(s): " + ("; ".join(msg) if msg else "ok"),
              flush=True)


if __name__ == "__main__":
    main()
