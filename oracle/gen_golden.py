"""TEST INFRASTRUCTURE ONLY -- regenerate tests/golden/ from the REAL reference.

Run in the build container (where /root/reference exists):

    make -C oracle && python -m oracle.gen_golden

It drives oracle/_ref/libref_rs.so (the unmodified lib/fec.cpp + lib/rs.cpp,
compiled by oracle/Makefile) and writes small data fixtures:

  kat_rs3_6.json        misc.cpp:335-361 known-answer test (RS(3,6) "aaa","bbb","ccc")
  matrices.npz          parity rows of fec_new's matrix for a (k,n) set, via rs_encode2
  encode_small.npz      parity for SplitMix64-seeded data, several (k,n,len)
  decode_small.npz      rs_decode2 results for erasure patterns, incl. non-codeword
                        inputs (random parity) that pin the lowest-k-survivors rule,
                        extra survivors, too-few survivors, and the pointer permutation
  full_hashes.json      sha256 over full-size C1 encode parity, C3 ragged parity, a
                        C2 non-codeword decode (pins the PRNG definitions too), and
                        the C4 rank slices 0, 3, 5, 7 of 8 over 2^20 groups (encode
                        parity + non-codeword decode), and per-group-checksum digests
                        of every range a bench.py rank owns at N = 1, 2, 4, 8
                        (python -m oracle.gen_golden --c4)

Inputs are regenerated from the PRNG definitions in oracle/cpu.py, so the fixtures
hold outputs (plus sha256 of inputs to pin the generator).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

from oracle.cpu import (DATA_SEED, ERASE_SEED, RAGGED_SEED, Oracle, Reference, erasures,
                        group_data, present_from_erasures, ragged_draw,
                        ragged_erasures)

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")

MATRIX_SET = [(1, 1), (1, 2), (1, 4), (2, 3), (2, 6), (3, 6), (4, 8), (10, 16), (20, 30),
              (16, 25), (7, 13), (127, 128), (128, 255), (200, 254), (64, 128), (2, 255),
              (254, 255), (255, 255), (100, 200), (1, 256), (256, 256), (32, 64)]
C3_STR = "1:3,2:4,10:6,20:10"

ENCODE_CASES = [  # (k, n, len, groups)
    (3, 6, 3, 2), (1, 4, 64, 3), (2, 6, 17, 3), (10, 16, 100, 3), (7, 13, 257, 2),
    (20, 30, 1, 5), (20, 30, 1250, 3), (20, 30, 31, 4), (16, 25, 1000, 1), (128, 255, 64, 1),
    (200, 254, 16, 1), (255, 255, 8, 1), (5, 5, 40, 2), (32, 64, 96, 1),
]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def layout(k, n, ln, ng, stride=None):
    s = stride or max(16, (ln + 15) // 16 * 16)
    buf = np.zeros((ng, n, s), np.uint8)
    buf[:, :k, :ln] = group_data(DATA_SEED, 0, ng, k, ln)
    return buf, s


def kat(ref: Reference):
    # misc.cpp:335-361: buffers of 100 B holding "aaa".."fff", rs_encode2(3,6,data,3),
    # then data[0]=0 and rs_decode2(3,6,data,3).
    buf = np.zeros((6, 100), np.uint8)
    for i, s in enumerate([b"aaa", b"bbb", b"ccc", b"ddd", b"eee", b"fff"]):
        buf[i, :3] = np.frombuffer(s, np.uint8)
    ref.encode_batch(3, 6, buf.reshape(-1), 600, 100, 3, 1)
    parity = [buf[i, :3].tobytes().hex() for i in range(3, 6)]
    rc, out = ref.decode_ptrs(3, 6, buf.reshape(-1), 100, 3, np.array([-1, 1, 2, 3, 4, 5]))
    shards = [buf[s, :3].tobytes().hex() if s >= 0 else None for s in out]
    return {"source": "misc.cpp:335-361", "k": 3, "n": 6, "size": 3,
            "data": ["616161", "626262", "636363"], "parity": parity,
            "decode_erase": [0], "decode_rc": int(rc), "decode_out_slots": out.tolist(),
            "decode_out_bytes": shards}


def encode_small(ref: Reference):
    d = {}
    for (k, n, ln, ng) in ENCODE_CASES:
        buf, s = layout(k, n, ln, ng)
        d[f"data_sha_{k}_{n}_{ln}_{ng}"] = np.frombuffer(
            bytes.fromhex(sha(buf[:, :k, :ln])), np.uint8)
        ref.encode_batch(k, n, buf.reshape(-1), n * s, s, ln, ng)
        d[f"parity_{k}_{n}_{ln}_{ng}"] = buf[:, k:, :ln].copy()
    return d


def decode_small(ref: Reference):
    """Cases: name -> (k, n, len, present[ng, n], codeword?)"""
    rng_cases = []
    k, n, ln = 20, 30, 1250
    ng = 6
    # uniform random 5-of-30 erasures, codeword input
    rng_cases.append(("c2_codeword", k, n, ln, present_from_erasures(
        erasures(ERASE_SEED, 0, ng, n, 5), n), True))
    # 5 data erasures (worst case), non-codeword parity (random bytes)
    rng_cases.append(("data5_noncodeword", k, n, ln, present_from_erasures(
        erasures(ERASE_SEED + 1, 0, ng, n, 5, limit=k), n), False))
    # every shard present, non-codeword: must use data as-is (no change)
    rng_cases.append(("all_present", k, n, ln, np.ones((2, n), np.uint8), False))
    # exactly k present: all 10 erasures within data, non-codeword
    rng_cases.append(("data10_noncodeword", k, n, ln, present_from_erasures(
        erasures(ERASE_SEED + 2, 0, 3, n, 10, limit=k), n), False))
    # 10 random erasures over 30, non-codeword
    rng_cases.append(("any10_noncodeword", k, n, ln, present_from_erasures(
        erasures(ERASE_SEED + 3, 0, 4, n, 10), n), False))
    # too few survivors -> -1
    rng_cases.append(("too_few", k, n, ln, present_from_erasures(
        erasures(ERASE_SEED + 4, 0, 2, n, 11), n), False))
    # parity-only erasures
    pres = np.ones((2, n), np.uint8); pres[:, 20:25] = 0
    rng_cases.append(("parity_only", k, n, ln, pres, False))
    # small / edge codes
    rng_cases.append(("rs3_6", 3, 6, 3, np.array([[0, 1, 1, 1, 1, 1], [0, 0, 1, 1, 0, 1],
                                                 [1, 0, 0, 0, 1, 1]], np.uint8), False))
    rng_cases.append(("rs1_4", 1, 4, 64, np.array([[0, 1, 1, 1], [0, 0, 0, 1]], np.uint8), False))
    rng_cases.append(("rs7_13_ragged_len", 7, 13, 257, present_from_erasures(
        erasures(ERASE_SEED + 5, 0, 3, 13, 6), 13), False))
    rng_cases.append(("rs128_255", 128, 255, 32, present_from_erasures(
        erasures(ERASE_SEED + 6, 0, 1, 255, 127), 255), False))
    rng_cases.append(("rs200_254", 200, 254, 16, present_from_erasures(
        erasures(ERASE_SEED + 7, 0, 1, 254, 54, limit=200), 254), False))
    rng_cases.append(("len0", 4, 8, 0, present_from_erasures(
        erasures(ERASE_SEED + 8, 0, 2, 8, 3), 8), False))
    d = {}
    for (name, k, n, ln, present, codeword) in rng_cases:
        ng = present.shape[0]
        s = max(16, (ln + 15) // 16 * 16)
        buf = np.zeros((ng, n, s), np.uint8)
        buf[:, :k, :ln] = group_data(DATA_SEED, 0, ng, k, ln)
        if codeword:
            ref.encode_batch(k, n, buf.reshape(-1), n * s, s, ln, ng)
        else:
            buf[:, k:, :ln] = group_data(DATA_SEED ^ 0xFFFF, 0, ng, n - k, ln)
        inp = buf.copy()
        # erased slots hold junk that must never be read
        for g in range(ng):
            for j in range(n):
                if not present[g, j]:
                    buf[g, j, :] = 0xA5
        status = ref.decode_batch(k, n, buf.reshape(-1), n * s, s, ln, ng, present)
        d[f"{name}__meta"] = np.array([k, n, ln, ng, int(codeword)], np.int64)
        d[f"{name}__present"] = present
        d[f"{name}__status"] = status
        d[f"{name}__input_sha"] = np.frombuffer(bytes.fromhex(sha(inp[:, :, :ln])), np.uint8)
        miss = [(g, j) for g in range(ng) if status[g] == 0 for j in range(k) if not present[g, j]]
        rec = np.stack([buf[g, j, :ln] for (g, j) in miss]) if miss else np.zeros((0, ln), np.uint8)
        d[f"{name}__recovered"] = rec  # recovered rows, (group, row) order, status 0 groups only
        d[f"{name}__data_out_sha"] = np.frombuffer(bytes.fromhex(sha(buf[:, :k, :ln])), np.uint8)
        # pointer permutation of rs_decode2 for group 0
        in_slot = np.where(present[0] > 0, np.arange(n), -1).astype(np.int32)
        b0 = inp[0].reshape(-1).copy()
        rc, out = ref.decode_ptrs(k, n, b0, s, ln, in_slot)
        d[f"{name}__ptr_rc"] = np.array([rc], np.int32)
        d[f"{name}__ptr_out"] = out
        d[f"{name}__ptr_bufs_sha"] = np.frombuffer(
            bytes.fromhex(sha(b0.reshape(n, s)[:, :ln])), np.uint8)
    return d


def full_hashes(ref: Reference, ora: Oracle, nthreads: int):
    res = {}
    # C1: RS(20,10), 1250 B, 65536 groups, device stride 1280 (only len bytes hashed)
    k, n, ln, G = 20, 30, 1250, 65536
    chunk = 4096
    hp = hashlib.sha256(); hd = hashlib.sha256()
    for g0 in range(0, G, chunk):
        buf = np.zeros((chunk, n, ln), np.uint8)
        buf[:, :k] = group_data(DATA_SEED, g0, chunk, k, ln)
        ref.encode_batch(k, n, buf.reshape(-1), n * ln, ln, ln, chunk, nthreads)
        hd.update(buf[:, :k].tobytes()); hp.update(buf[:, k:].tobytes())
    res["c1_encode"] = {"k": k, "n": n, "len": ln, "groups": G, "seed": DATA_SEED,
                        "data_sha256": hd.hexdigest(), "parity_sha256": hp.hexdigest()}
    # C2 non-codeword decode: random parity, 5 erasures/group over 30 -> sha of data rows
    hx = hashlib.sha256()
    for g0 in range(0, G, chunk):
        buf = np.zeros((chunk, n, ln), np.uint8)
        buf[:, :k] = group_data(DATA_SEED, g0, chunk, k, ln)
        buf[:, k:] = group_data(DATA_SEED ^ 0xFFFF, g0, chunk, n - k, ln)
        pres = present_from_erasures(erasures(ERASE_SEED, g0, chunk, n, 5), n)
        st = ref.decode_batch(k, n, buf.reshape(-1), n * ln, ln, ln, chunk, pres,
                              True, nthreads)
        assert (st == 0).all()
        hx.update(buf[:, :k].tobytes())
    res["c2_decode_noncodeword"] = {"k": k, "n": n, "len": ln, "groups": G,
                                    "erasures": 5, "erase_seed": ERASE_SEED,
                                    "parity_seed": DATA_SEED ^ 0xFFFF,
                                    "data_out_sha256": hx.hexdigest()}
    # C3 ragged encode: k~U{1..20}, m = rs_from_str(C3_STR), len~U[64..1250]
    tab = ora.rs_from_str(C3_STR)
    ty = np.array([y for (_, y) in tab], np.int64)
    kk, mm, ll = ragged_draw(RAGGED_SEED, 0, G, ty)
    hr = hashlib.sha256()
    for g in range(G):
        k_, m_, l_ = int(kk[g]), int(mm[g]), int(ll[g])
        buf = np.zeros((k_ + m_, l_), np.uint8)
        buf[:k_] = group_data(DATA_SEED, g, 1, k_, l_)[0]
        ref.encode_batch(k_, k_ + m_, buf.reshape(-1), 0, l_, l_, 1)
        hr.update(buf[k_:].tobytes())
    res["c3_ragged_encode"] = {"fec": C3_STR, "groups": G, "ragged_seed": RAGGED_SEED,
                               "kmax": 20, "len_min": 64, "len_max": 1250,
                               "sum_payload": int((kk * ll).sum()),
                               "sum_parity": int((mm * ll).sum()),
                               "parity_sha256": hr.hexdigest()}
    res["c3_ragged_decode"] = c3_ragged_decode(ref, ora)
    return res


def c3_ragged_decode(ref: Reference, ora: Oracle):
    """C3 ragged decode, non-codeword: group g's data rows are the DATA_SEED
    stream, its parity rows the DATA_SEED ^ 0xFFFF stream (not a codeword, so
    the output pins which survivors rs_decode uses), it loses min(5, m) of its
    n shards (ragged_erasures), the reference rs_decode2 rebuilds it; the
    digest covers every group's k data rows (len bytes each) in order."""
    tab = ora.rs_from_str(C3_STR)
    ty = np.array([y for (_, y) in tab], np.int64)
    G = 65536
    kk, mm, ll = ragged_draw(RAGGED_SEED, 0, G, ty)
    pres = ragged_erasures(ERASE_SEED, 0, kk + mm, mm, 5)
    h = hashlib.sha256()
    rebuilt = 0
    for g in range(G):
        k_, m_, l_ = int(kk[g]), int(mm[g]), int(ll[g])
        n_ = k_ + m_
        buf = np.zeros((n_, l_), np.uint8)
        buf[:k_] = group_data(DATA_SEED, g, 1, k_, l_)[0]
        buf[k_:] = group_data(DATA_SEED ^ 0xFFFF, g, 1, m_, l_)[0]
        p = pres[g:g + 1, :n_]
        st = ref.decode_batch(k_, n_, buf.reshape(-1), 0, l_, l_, 1, p, True, 1)
        assert st[0] == 0
        rebuilt += int((p[0, :k_] == 0).sum())
        h.update(buf[:k_].tobytes())
    return {"fec": C3_STR, "groups": G, "ragged_seed": RAGGED_SEED, "erase_seed": ERASE_SEED,
            "erasures": 5, "parity_seed": DATA_SEED ^ 0xFFFF, "rebuilt_rows": rebuilt,
            "data_out_sha256": h.hexdigest()}


C4_GROUPS = 1 << 20
C4_WORLD = 8
C4_RANKS = (0, 3, 5, 7)
C4_WORLDS = (1, 2, 4, 8)
C4_WEAK = 65536  # bench.py --scaling weak / N = 1: groups per rank


def c4_ranges():
    """Every group range a bench.py rank can own over the C4 stream: the
    strong splits of 2^20 groups over 1/2/4/8 ranks and the weak 65,536-group
    blocks of ranks 0..7 (block 0 is the N = 1 C1+C2 batch)."""
    rs = set()
    for w in C4_WORLDS:
        for r in range(w):
            rs.add((C4_GROUPS * r // w, C4_GROUPS * (r + 1) // w))
    for r in range(8):
        rs.add((r * C4_WEAK, (r + 1) * C4_WEAK))
    return sorted(rs)


def c4_rank_slices(ref: Reference, nthreads: int):
    """C4 (RS(20,10), 1250 B, 2^20 groups; global group ids drive the PRNG
    streams), run through the reference in one pass over all groups:
      ranks[r]        for ranks 0, 3, 5, 7 of 8, the slice [g0, g1) =
                      shard.strong_range(r, 8, 2^20) as one rank encodes and
                      decodes it:
        parity_sha256   rs_encode2 parity of the slice's DATA_SEED data;
        data_out_sha256 rs_decode2 of the non-codeword slice (DATA_SEED data,
                        DATA_SEED ^ 0xFFFF parity, 5 erasures per group from
                        ERASE_SEED), digest of the k data rows (len bytes each);
      ranges["g0-g1"] for every range of c4_ranges(): sha256 over the per-group
                      checksums (oracle.cpu.group_hashes) of the same parity
                      rows ("parity_gsum") and decoded data rows
                      ("data_out_gsum") -- what bench.py's ranks check their
                      slices against after the timed region.
    Groups are independent (connection.h:244-245), so each slice's digest is
    what rank r of an N-GPU job must produce."""
    from oracle.cpu import group_hashes
    k, n, ln = 20, 30, 1250
    chunk = 8192
    out = {"k": k, "n": n, "len": ln, "groups": C4_GROUPS, "world": C4_WORLD,
           "seed": DATA_SEED, "parity_seed": DATA_SEED ^ 0xFFFF, "erase_seed": ERASE_SEED,
           "erasures": 5, "checksum": "oracle.cpu.group_hashes / udpspeeder_amd.synth.group_hashes_dev",
           "ranks": {}, "ranges": {}}
    bounds = {r: (C4_GROUPS * r // C4_WORLD, C4_GROUPS * (r + 1) // C4_WORLD) for r in C4_RANKS}
    sh = {r: (hashlib.sha256(), hashlib.sha256()) for r in C4_RANKS}
    hpar = np.empty(C4_GROUPS, np.uint64)
    hdat = np.empty(C4_GROUPS, np.uint64)
    for c0 in range(0, C4_GROUPS, chunk):
        m = min(chunk, C4_GROUPS - c0)
        buf = np.zeros((m, n, ln), np.uint8)
        buf[:, :k] = group_data(DATA_SEED, c0, m, k, ln)
        ref.encode_batch(k, n, buf.reshape(-1), n * ln, ln, ln, m, nthreads)
        hpar[c0:c0 + m] = group_hashes(buf[:, k:])
        owner = [r for r, (a, b) in bounds.items() if a <= c0 < b]
        if owner:
            sh[owner[0]][0].update(buf[:, k:].tobytes())
        buf[:, k:] = group_data(DATA_SEED ^ 0xFFFF, c0, m, n - k, ln)
        pres = present_from_erasures(erasures(ERASE_SEED, c0, m, n, 5), n)
        st = ref.decode_batch(k, n, buf.reshape(-1), n * ln, ln, ln, m, pres, True, nthreads)
        assert (st == 0).all()
        hdat[c0:c0 + m] = group_hashes(buf[:, :k])
        if owner:
            sh[owner[0]][1].update(buf[:, :k].tobytes())
        if c0 % (chunk * 16) == 0:
            print("c4", c0, flush=True)
    for r in C4_RANKS:
        g0, g1 = bounds[r]
        out["ranks"][str(r)] = {"g0": g0, "g1": g1, "parity_sha256": sh[r][0].hexdigest(),
                                "data_out_sha256": sh[r][1].hexdigest()}
    dig = lambda h: hashlib.sha256(np.ascontiguousarray(h, dtype="<u8").tobytes()).hexdigest()
    for g0, g1 in c4_ranges():
        out["ranges"][f"{g0}-{g1}"] = {"parity_gsum": dig(hpar[g0:g1]),
                                       "data_out_gsum": dig(hdat[g0:g1])}
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    ref = Reference()
    ora = Oracle()
    if sys.argv[1:] == ["--c4"]:  # add/refresh only the C4 rank-slice digests
        path = os.path.join(OUT, "full_hashes.json")
        full = json.load(open(path))
        full["c4_rank_slices"] = c4_rank_slices(ref, os.cpu_count() or 1)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        print("c4_rank_slices written to", path)
        return
    if sys.argv[1:] == ["--c3-decode"]:  # add/refresh only the C3 decode digest
        path = os.path.join(OUT, "full_hashes.json")
        full = json.load(open(path))
        full["c3_ragged_decode"] = c3_ragged_decode(ref, ora)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        print("c3_ragged_decode written to", path)
        return
    with open(os.path.join(OUT, "kat_rs3_6.json"), "w") as f:
        json.dump(kat(ref), f, indent=1)
    mats = {f"{k}_{n}": ref.enc_matrix(k, n)[k:] for (k, n) in MATRIX_SET}
    mats["c3_table"] = np.array(ora.rs_from_str(C3_STR), np.int64)
    np.savez_compressed(os.path.join(OUT, "matrices.npz"), **mats)
    np.savez_compressed(os.path.join(OUT, "encode_small.npz"), **encode_small(ref))
    np.savez_compressed(os.path.join(OUT, "decode_small.npz"), **decode_small(ref))
    full = full_hashes(ref, ora, os.cpu_count() or 1)
    full["c4_rank_slices"] = c4_rank_slices(ref, os.cpu_count() or 1)
    with open(os.path.join(OUT, "full_hashes.json"), "w") as f:
        json.dump(full, f, indent=1)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
