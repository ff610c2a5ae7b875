#!/usr/bin/env python3
"""Build-time generator of the bit-sliced RS encoders (gen/bitslice_codes.inc).

For a fixed code (k, n) the encoder is a fixed GF(2)-linear map from the 8k
input bit-planes to the 8m output bit-planes: multiplication by a constant c
is the 8x8 bit matrix M_c[u][t] = bit u of (c * 2^t) (GF(2^8) multiplication
is linear over GF(2)).  The matrix of the code is fec_new's systematic
Vandermonde matrix (lib/fec.cpp:665-720), computed here from scratch.

Each lane holds 32 bytes of every shard as 8 dwords; an in-register 8x8 bit
transpose (per byte lane) turns them into 8 bit-planes, so one 32-bit XOR
adds 32 byte positions at once.  The XOR network is emitted with the "four
Russians" split: per input shard, the XOR combinations of planes {0..3} and
{4..7} that the outputs need are formed once, then every output plane takes
at most one combination from each half -- one 3-input XOR (v_bitop3_b32) per
(output plane, input shard).

The emitted function is __host__ __device__ and templated on an IO policy,
so the same generated network is unit-tested on the CPU (tests/) and runs in
the HIP kernels (bitslice.hip).
"""
from __future__ import annotations

import argparse
import os
import sys

# ---------------------------------------------------------------- GF(2^8), 0x11D
EXP = [0] * 512
LOG = [0] * 256
_v = 1
for _i in range(255):
    EXP[_i] = _v
    LOG[_v] = _i
    _v <<= 1
    if _v & 0x100:
        _v ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def gmul(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return EXP[LOG[a] + LOG[b]]


def ginv(a: int) -> int:
    return EXP[(255 - LOG[a]) % 255]


def invert(mat):
    k = len(mat)
    a = [row[:] + [1 if i == j else 0 for j in range(k)] for i, row in enumerate(mat)]
    for c in range(k):
        p = next(r for r in range(c, k) if a[r][c])
        a[c], a[p] = a[p], a[c]
        s = ginv(a[c][c])
        a[c] = [gmul(s, x) for x in a[c]]
        for r in range(k):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [x ^ gmul(f, y) for x, y in zip(a[r], a[c])]
    return [row[k:] for row in a]


def enc_matrix(k: int, n: int):
    """Parity rows (n-k) x k of fec_new(k, n)."""
    v = [[0] * k for _ in range(n)]
    v[0][0] = 1
    for r in range(1, n):
        for c in range(k):
            v[r][c] = EXP[((r - 1) * c) % 255]
    inv = invert([row[:] for row in v[:k]])
    out = []
    for r in range(k, n):
        out.append([0] * k)
        for c in range(k):
            acc = 0
            for i in range(k):
                acc ^= gmul(v[r][i], inv[i][c])
            out[-1][c] = acc
    return out


def bitmat(c: int):
    """M[u][t] = bit u of c * 2^t."""
    cols = [gmul(c, 1 << t) for t in range(8)]
    return [[(cols[t] >> u) & 1 for t in range(8)] for u in range(8)]


# ---------------------------------------------------------------- emitter
RING = int(os.environ.get("BS_RING", "4"))  # raw-load ring: shard j+RING is requested while shard j is computed


MAX_ROWS = int(os.environ.get("BS_MAX_ROWS", "10"))  # parity rows per pass: 8 accumulators each (at 12 rows the 168-VGPR budget spills)


def row_blocks(m: int):
    """Passes over the input for m parity rows: ceil(m / MAX_ROWS) blocks of
    near-equal size.  Every pass reloads the k input shards."""
    nb = max(1, (m + MAX_ROWS - 1) // MAX_ROWS)
    bs = (m + nb - 1) // nb
    return [(b * bs, min(m, (b + 1) * bs)) for b in range(nb) if b * bs < m]


def emit_code(k: int, n: int):
    m = n - k
    P = enc_matrix(k, n)
    L = []
    nxor = 0
    blocks = row_blocks(m)
    L.append(f"// RS(k={k}, n={n}): {8 * m} output planes <- {8 * k} input planes")
    L.append(f"template <class IO>")
    L.append(f"__host__ __device__ __forceinline__ void bs_code_{k}_{n}(IO &io) {{")
    for (r0, r1) in blocks:
        ind = "    " if len(blocks) == 1 else "        "
        if len(blocks) > 1:
            L.append(f"    {{  // parity rows {r0}..{r1 - 1}")
        nxor += emit_block(L.append, ind, k, P, r0, r1)
        if len(blocks) > 1:
            L.append(f"    }}")
            L.append(f"    BS_SCHED_BARRIER();")
    L.append(f"}}  // {nxor} XOR ops")
    return "\n".join(L), nxor


def emit_block(w0, ind, k, P, r0, r1):
    """One pass: load every input shard once, accumulate parity rows r0..r1-1."""
    def w(line):
        w0(ind + line)
    for i in range(r0, r1):
        w("uint32_t " + ", ".join(f"o{i}_{u} = 0" for u in range(8)) + ";")
    nxor = emit_shards(w, P, r0, r1, 0, k)
    for i in range(r0, r1):
        emit_store(w, k, i)
    return nxor


def emit_store(w, k, i):
    w(f"{{")
    w(f"    uint32_t q[8] = {{" + ", ".join(f"o{i}_{u}" for u in range(8)) + "};")
    w(f"    bs_transpose8(q);")
    w(f"    io.store({k + i}, q);")
    w(f"}}")


def emit_shards(w, P, r0, r1, j0, j1):
    """Input shards j0..j1-1 through a RING-deep raw-load ring, accumulated into
    parity rows r0..r1-1 (o<row>_<plane>, declared by the caller)."""
    nxor = 0
    R = min(RING, j1 - j0)
    w("uint32_t " + ", ".join(f"rb{r}[8]" for r in range(R)) + ";")
    for r in range(R):
        w(f"io.load({j0 + r}, rb{r});")
    for j in range(j0, j1):
        w(f"{{  // input shard {j}")
        w(f"    uint32_t (&p)[8] = rb{(j - j0) % R};")
        w(f"    bs_transpose8(p);")
        need_lo, need_hi = {}, {}
        terms = {}
        for i in range(r0, r1):
            M = bitmat(P[i][j])
            for u in range(8):
                lo = sum(M[u][t] << t for t in range(4))
                hi = sum(M[u][t + 4] << t for t in range(4))
                terms[(i, u)] = (lo, hi)
                if lo:
                    need_lo[lo] = 1
                if hi:
                    need_hi[hi] = 1

        # combination names: single planes are p[t]; multi-plane masks get a temp
        def build(needed, base, tag):
            nonlocal nxor
            names = {}
            for t in range(4):
                names[1 << t] = f"p[{base + t}]"

            def get(mm):
                # split off the highest plane; build the rest recursively
                nonlocal nxor
                if mm in names:
                    return names[mm]
                hb = mm.bit_length() - 1
                rest = mm & ~(1 << hb)
                a = get(rest)
                nm = f"{tag}{mm}"
                w(f"    const uint32_t {nm} = {a} ^ p[{base + hb}];")
                nxor += 1
                names[mm] = nm
                return nm

            for mask in sorted(needed, key=lambda x: bin(x).count("1")):
                get(mask)
            return names

        lo_names = build(need_lo, 0, "l")
        hi_names = build(need_hi, 4, "h")
        for i in range(r0, r1):
            for u in range(8):
                lo, hi = terms[(i, u)]
                a = lo_names[lo] if lo else None
                b = hi_names[hi] if hi else None
                acc = f"o{i}_{u}"
                if a and b:
                    w(f"    BS_ACC3({acc}, {a}, {b});")
                    nxor += 1
                elif a or b:
                    w(f"    BS_ACC2({acc}, {a or b});")
                    nxor += 1
        if j + R < j1:
            w(f"    io.load({j + R}, rb{(j - j0) % R});")
        w(f"}}")
        w(f"BS_SCHED_BARRIER();")
    return nxor


# ---------------------------------------------------------------- split-k form
# Two waves per 128-column chunk: wave h accumulates ALL m parity rows over its
# half of the input shards (h = 0: shards 0..ka-1, h = 1: ka..k-1), hands the
# partial sums of the partner's rows over LDS (x.send / x.sync / x.recv), adds
# the partner's partials of its own rows, and stores those (h = 0: rows
# 0..mh-1, h = 1: mh..m-1).  Each wave then touches half the shard rows of the
# chunk: the chip's concurrent HBM footprint per wave halves
# (scripts/probes/mix_probe.hip "split-k": 3 % faster access pattern).
SPLIT_MAX_ROWS = 5  # rows handed over per wave: the kernel's LDS exchange is sized for this


def split_ok(k: int, n: int) -> bool:
    m = n - k
    return k >= 10 and 2 <= m <= 2 * SPLIT_MAX_ROWS


def emit_split(k: int, n: int):
    m = n - k
    P = enc_matrix(k, n)
    ka, mh = (k + 1) // 2, (m + 1) // 2
    L = [f"// RS(k={k}, n={n}) split-k: shards 0..{ka - 1} | {ka}..{k - 1}, rows 0..{mh - 1} | {mh}..{m - 1}",
         "template <class IO, class XCH>",
         f"__device__ __forceinline__ void bs_split_{k}_{n}(IO &io, uint32_t h, XCH &x) {{"]
    nxor = 0
    for h, (j0, j1), (own0, own1), (oth0, oth1) in (
            (0, (0, ka), (0, mh), (mh, m)), (1, (ka, k), (mh, m), (0, mh))):
        L.append("    if (h == 0) {" if h == 0 else "    } else {")

        def w(line):
            L.append("        " + line)
        for i in range(m):
            w("uint32_t " + ", ".join(f"o{i}_{u} = 0" for u in range(8)) + ";")
        nxor += emit_shards(w, P, 0, m, j0, j1)
        for r, i in enumerate(range(oth0, oth1)):
            w(f"x.send({r}, " + ", ".join(f"o{i}_{u}" for u in range(8)) + ");")
        w("x.sync();")
        for r, i in enumerate(range(own0, own1)):
            w(f"x.recv({r}, " + ", ".join(f"o{i}_{u}" for u in range(8)) + ");")
        for i in range(own0, own1):
            emit_store(w, k, i)
    L.append("    }")
    L.append(f"}}  // {nxor} XOR ops + {8 * m} exchange XORs")
    return "\n".join(L), nxor


def default_codes():
    codes = set()
    for x in range(1, 21):
        codes.add((x, x + 10))           # UDPspeeder default -f 20:10 (misc.cpp:57)
    c3 = [(1, 3), (2, 4), (3, 5), (4, 5), (5, 5), (6, 5), (7, 6), (8, 6), (9, 6), (10, 6),
          (11, 7), (12, 7), (13, 8), (14, 8), (15, 8), (16, 9), (17, 9), (18, 10), (19, 10),
          (20, 10)]                      # rs_from_str("1:3,2:4,10:6,20:10")
    for x, y in c3:
        codes.add((x, x + y))
    return sorted(codes)


def embed(out, specs):
    here = os.path.dirname(os.path.abspath(__file__))
    parts = ["// GENERATED by gen_bitslice.py --embed -- do not edit."]
    for spec in specs:
        path, name = spec.rsplit(":", 1)
        txt = open(os.path.join(here, path)).read()
        txt = "\n".join(l for l in txt.split("\n") if l.strip() != "#pragma once") + "\n"
        assert ')rsmi"' not in txt
        parts.append(f'static const char {name}[] = R"rsmi({txt})rsmi";')
    txt = "\n".join(parts) + "\n"
    if not (os.path.exists(out) and open(out).read() == txt):
        with open(out, "w") as f:
            f.write(txt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                  "gen", "bitslice_codes.inc"))
    ap.add_argument("--codes", default="", help="k:n,k:n,... (default: built-in hot set)")
    ap.add_argument("--embed", nargs="+", metavar="OUT FILE:NAME",
                    help="write FILEs as C++ string constants NAME into OUT (the device "
                         "headers bitslice_rtc.cpp hands to hipRTC)")
    args = ap.parse_args()
    if args.embed:
        return embed(args.embed[0], args.embed[1:])
    codes = default_codes() if not args.codes else \
        [tuple(int(v) for v in c.split(":")) for c in args.codes.split(",")]
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    parts = ["// GENERATED by gen_bitslice.py -- do not edit.",
             "// Bit-sliced XOR networks for the hot (k,n) codes of fec_new's matrix.",
             f"#define BS_NUM_CODES {len(codes)}"]
    stats = []
    for (k, n) in codes:
        src, nx = emit_code(k, n)
        parts.append(src)
        stats.append((k, n, nx))
    parts.append("#define BS_FOR_EACH_CODE(X) \\")
    parts.append(" \\\n".join(f"    X({k}, {n})" for (k, n) in codes))
    split = [(k, n) for (k, n) in codes if split_ok(k, n)]
    parts.append("#ifdef __HIPCC__  // device-only: the split form synchronises a wave pair")
    for (k, n) in split:
        parts.append(emit_split(k, n)[0])
    parts.append("#define BS_FOR_EACH_SPLIT(X) \\")
    parts.append(" \\\n".join(f"    X({k}, {n})" for (k, n) in split))
    parts.append("#endif")
    parts.append("")
    txt = "\n".join(parts) + "\n"
    if os.path.exists(args.out) and open(args.out).read() == txt:
        return
    with open(args.out, "w") as f:
        f.write(txt)
    for k, n, nx in stats:
        print(f"  bs_code_{k}_{n}: {nx} xor ops ({nx / (32 * k):.2f} per input byte)",
              file=sys.stderr)


if __name__ == "__main__":
    main()
