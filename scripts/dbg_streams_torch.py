"""Debug: the access pattern of dbg_streams.py (two streams, per stream: write
rows k..n-1 from rows 0..k-1, overwrite erased rows with 0x77, rebuild them)
done with torch ops only, so no librsmi kernel runs.  Wrong bytes here would
point at the platform, not at the codec."""
import sys

import numpy as np
import torch


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    k, n, G, S = 20, 30, 2048, 1280
    gpu = torch.device("cuda:0")
    for rep in range(reps):
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        g = torch.Generator(device="cpu").manual_seed(rep)
        clean = [torch.randint(0, 256, (G, n, S), dtype=torch.uint8, generator=g).to(gpu) for _ in range(2)]
        for c in clean:  # "parity": rows k.. = xor of rolled data rows
            c[:, k:] = c[:, :n - k] ^ c[:, k - (n - k):k]
        ts = [torch.zeros((G, n, S), dtype=torch.uint8, device=gpu) for _ in range(2)]
        for t, c in zip(ts, clean):
            t[:, :k] = c[:, :k]
        pres = []
        for i in range(2):
            p = np.ones((G, n), np.uint8)
            rng = np.random.default_rng(7 + i + 100 * rep)
            for r in range(G):
                p[r, rng.choice(n, 5, replace=False)] = 0
            pres.append(torch.from_numpy(p).to(gpu))
        torch.cuda.synchronize()
        for _ in range(3):
            for t, s, p, c in zip(ts, (s1, s2), pres, clean):
                with torch.cuda.stream(s):
                    t[:, k:] = t[:, :n - k] ^ t[:, k - (n - k):k]
                    m = (p == 0).unsqueeze(-1)
                    t.masked_fill_(m, 0x77)
                    t.copy_(torch.where(m, c, t))
        torch.cuda.synchronize()
        msg = []
        for i, (t, c) in enumerate(zip(ts, clean)):
            bad = (t != c).any(dim=2).nonzero()
            if len(bad):
                msg.append(f"t{i}: {len(bad)} bad rows, first {bad[0].tolist()}")
        print(f"torch rep {rep}: " + ("; ".join(msg) if msg else "ok"), flush=True)


if __name__ == "__main__":
    main()
