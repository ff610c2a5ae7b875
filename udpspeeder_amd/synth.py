"""Synthetic workload definitions for the bench and tests.

All draws are counter-based SplitMix64: word w of stream (seed, g) is
``mix((seed ^ g) + (w + 1) * 0x9E3779B97F4A7C15)``.

* data bytes (C1-C4): generated on the GPU by ``rs.fill_data``;
* erasure patterns (C2): e distinct indices per group from a partial
  Fisher-Yates over range(limit) driven by the group's stream;
* ragged mix (C3): k ~ U{1..kmax}, m from the ``-f`` table, len ~ U[lmin, lmax].
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
DATA_SEED = 0x5EEDC0DE
ERASE_SEED = 0xE7A5E5EED
RAGGED_SEED = 0x7A66ED
C3_FEC = "1:3,2:4,10:6,20:10"


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def stream_words(seed: int, g0: int, ng: int, nwords: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        s0 = np.uint64(seed) ^ np.arange(g0, g0 + ng, dtype=np.uint64)
        w = np.arange(1, nwords + 1, dtype=np.uint64) * GAMMA
        return _mix(s0[:, None] + w[None, :])


def erasure_present(seed: int, g0: int, ng: int, n: int, e: int, limit: int = 0) -> np.ndarray:
    """[ng, n] uint8 present flags with e erasures per group."""
    lim = limit or n
    r = stream_words(seed, g0, ng, e)
    perm = np.tile(np.arange(lim, dtype=np.int64), (ng, 1))
    rows = np.arange(ng)
    for i in range(e):
        pick = i + (r[:, i] % np.uint64(lim - i)).astype(np.int64)
        a = perm[rows, i].copy()
        perm[rows, i] = perm[rows, pick]
        perm[rows, pick] = a
    pres = np.ones((ng, n), np.uint8)
    pres[rows[:, None], perm[:, :e]] = 0
    return pres


def ragged_erasures(seed: int, g0: int, ns, ms, emax: int = 5) -> np.ndarray:
    """[ng, 256] uint8 present flags for a ragged batch: group i (id g0 + i)
    loses min(emax, m_i) distinct shards drawn from range(n_i) by a partial
    Fisher-Yates on its stream (as erasure_present, with per-group n); flags
    at and beyond n_i are 0."""
    ns = np.asarray(ns, np.int64)
    ms = np.asarray(ms, np.int64)
    ng = len(ns)
    e = np.minimum(emax, ms)
    r = stream_words(seed, g0, ng, emax)
    perm = np.tile(np.arange(256, dtype=np.int64), (ng, 1))
    rows = np.arange(ng)
    for i in range(emax):
        act = i < e
        span = np.maximum(ns - i, 1).astype(np.uint64)
        pick = np.where(act, i + (r[:, i] % span).astype(np.int64), i)
        a = perm[rows, i].copy()
        perm[rows, i] = perm[rows, pick]
        perm[rows, pick] = a
    pres = (np.arange(256)[None, :] < ns[:, None]).astype(np.uint8)
    for i in range(emax):
        act = i < e
        pres[rows[act], perm[act, i]] = 0
    return pres


HASH_SEED = 0xC4C4D16E57


def hash_weights(nbytes: int) -> np.ndarray:
    """Odd uint64 weights of the per-group checksum: w_j = mix(HASH_SEED +
    (j + 1) * GAMMA) | 1 for byte j of a group's rows (row-major)."""
    with np.errstate(over="ignore"):
        j = np.arange(1, nbytes + 1, dtype=np.uint64) * GAMMA
        return _mix(np.uint64(HASH_SEED) + j) | np.uint64(1)


def group_hashes_dev(rows, chunk: int = 4096) -> np.ndarray:
    """Per-group checksum of a [G, R, L] uint8 tensor (any device, any
    strides): h_g = sum_j w_j * byte_j mod 2^64 over the group's R*L bytes.
    Every single-byte change moves h_g (odd weights); the digest of a range is
    sha256 over its h_g (``hashes_digest``).  The golden side restates it in
    numpy (oracle/cpu.py ``group_hashes``) from the reference's own bytes, so a
    rank checks its whole slice after the timed region by moving 8 B per group
    off the device instead of the slice itself."""
    import torch
    G, R, L = rows.shape
    w = torch.from_numpy(hash_weights(R * L).view(np.int64)).to(rows.device)
    out = torch.empty(G, dtype=torch.int64, device=rows.device)
    for c in range(0, G, chunk):
        b = rows[c:c + chunk].reshape(-1, R * L).to(torch.int64)
        out[c:c + chunk] = (b * w).sum(dim=1)  # int64 arithmetic wraps mod 2^64
    return out.cpu().numpy().view(np.uint64)


def hashes_digest(h) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(h, dtype="<u8").tobytes()).hexdigest()


def present_bits(flags) -> np.ndarray:
    """[ng, <=256] present flags -> the ragged decode's [ng, 8] uint32 masks
    (bit j % 32 of word j / 32 = shard j received)."""
    f = np.zeros((len(flags), 256), np.uint8)
    fl = np.asarray(flags, np.uint8)
    f[:, :fl.shape[1]] = fl != 0
    return np.packbits(f, axis=1, bitorder="little").view("<u4").reshape(-1, 8).copy()


def ragged_mix(seed: int, g0: int, ng: int, table_y, kmax: int = 20, lmin: int = 64,
               lmax: int = 1250):
    """(k, m, len) int64 arrays for the C3 ragged batch."""
    ty = np.asarray(table_y, np.int64)
    r = stream_words(seed, g0, ng, 2)
    k = 1 + (r[:, 0] % np.uint64(kmax)).astype(np.int64)
    ln = lmin + (r[:, 1] % np.uint64(lmax - lmin + 1)).astype(np.int64)
    return k, ty[k - 1], ln
