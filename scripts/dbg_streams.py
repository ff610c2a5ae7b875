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
    k, n, ln, G = 20, 30, 1250, 2048
    gpu = torch.device("cuda:0")
    orc = Oracle()
    lib = os.path.basename(os.environ.get("RSMI_LIB", "default"))
    for rep in range(reps):
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        if not two:
            s2 = s1
        ts = [torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu) for _ in range(2)]
        for i, t in enumerate(ts):
            u.fill_data(t, k, ln, 100 + i)
        torch.cuda.synchronize()
        ref = [t.cpu().numpy() for t in ts]
        pres = [torch.from_numpy(synth.erasure_present(7 + i, 0, G, n, 5)).to(gpu) for i in range(2)]
        for _ in range(3):
            for t, s, p in zip(ts, (s1, s2), pres):
                with torch.cuda.stream(s):
                    u.encode(t, k, n, ln)
                    t.masked_fill_((p == 0).unsqueeze(-1), 0x77)
                    u.decode(t, p, k, n, ln)
        torch.cuda.synchronize()
        msg = []
        for i, (t, r) in enumerate(zip(ts, ref)):
            orc.encode_batch(k, n, r.reshape(-1), n * 1280, 1280, ln, G)
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
        print(f"{lib} rep {rep} {'two' if two else 'one'} stream(s): " + ("; ".join(msg) if msg else "ok"),
              flush=True)


if __name__ == "__main__":
    main()
