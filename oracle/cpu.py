"""TEST INFRASTRUCTURE ONLY -- ctypes bindings for the CPU checkers.

* ``Oracle``  -> ``oracle/librsoracle.so``: our plain-C restatement of
  lib/fec.cpp + lib/rs.cpp (see rs_oracle.c for per-function citations).
* ``Reference`` -> ``oracle/_ref/libref_rs.so``: the unmodified reference
  lib/{fec,rs}.cpp compiled from /root/reference by oracle/Makefile, plus our
  batch driver (ref_driver.cpp).  Present only where it was built.

Also the synthetic-input definitions shared by tests, golden generation and the
bench's CPU leg (SplitMix64 byte streams, erasure draws, the C3 ragged mix), in
numpy.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product package never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "librsoracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_rs.so")

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

DATA_SEED = 0x5EEDC0DE
ERASE_SEED = 0xE7A5E5EED
RAGGED_SEED = 0x7A66ED


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def splitmix_words(seed: int, groups: np.ndarray, nwords: int) -> np.ndarray:
    """[len(groups), nwords] uint64: word w of group g's stream =
    mix((seed ^ g) + (w+1)*GAMMA)."""
    with np.errstate(over="ignore"):
        s0 = np.uint64(seed) ^ groups.astype(np.uint64)
        w = (np.arange(1, nwords + 1, dtype=np.uint64) * GAMMA)
        return _mix(s0[:, None] + w[None, :])


def group_data(seed: int, g0: int, ng: int, k: int, length: int) -> np.ndarray:
    """Data shards of groups g0..g0+ng-1 as [ng, k, length] uint8.  Byte q of a
    group's k*length data bytes (shard-major) is byte q%8 of stream word q//8."""
    nbytes = k * length
    nwords = (nbytes + 7) // 8
    words = splitmix_words(seed, np.arange(g0, g0 + ng, dtype=np.uint64), nwords)
    b = words.view(np.uint8).reshape(ng, nwords * 8)[:, :nbytes]
    return b.reshape(ng, k, length)


def erasures(seed: int, g0: int, ng: int, n: int, e: int, limit: int | None = None) -> np.ndarray:
    """[ng, e] erased shard indices per group: partial Fisher-Yates over
    range(limit or n) driven by words mix((seed^g)+(i+1)*GAMMA)."""
    lim = n if limit is None else limit
    r = splitmix_words(seed, np.arange(g0, g0 + ng, dtype=np.uint64), e)
    perm = np.tile(np.arange(lim, dtype=np.int64), (ng, 1))
    rows = np.arange(ng)
    for i in range(e):
        pick = i + (r[:, i] % np.uint64(lim - i)).astype(np.int64)
        a = perm[rows, i].copy()
        perm[rows, i] = perm[rows, pick]
        perm[rows, pick] = a
    return perm[:, :e]


def ragged_erasures(seed: int, g0: int, ns: np.ndarray, ms: np.ndarray, emax: int = 5) -> np.ndarray:
    """C3 decode erasures: [ng, 256] present flags; group g0+i loses min(emax,
    m_i) distinct shards, a partial Fisher-Yates over range(n_i) driven by
    words mix((seed^g)+(i+1)*GAMMA); flags at and beyond n_i are 0."""
    ns = np.asarray(ns, np.int64)
    ms = np.asarray(ms, np.int64)
    ng = len(ns)
    out = np.zeros((ng, 256), np.uint8)
    r = splitmix_words(seed, np.arange(g0, g0 + ng, dtype=np.uint64), emax) if emax else None
    for g in range(ng):
        n, e = int(ns[g]), int(min(emax, ms[g]))
        perm = list(range(n))
        for i in range(e):
            pick = i + int(r[g, i] % np.uint64(n - i))
            perm[i], perm[pick] = perm[pick], perm[i]
        out[g, :n] = 1
        out[g, perm[:e]] = 0
    return out


def present_from_erasures(er: np.ndarray, n: int) -> np.ndarray:
    p = np.ones((er.shape[0], n), dtype=np.uint8)
    p[np.arange(er.shape[0])[:, None], er] = 0
    return p


def ragged_draw(seed: int, g0: int, ng: int, table_y: np.ndarray,
                kmax: int = 20, lmin: int = 64, lmax: int = 1250):
    """C3 ragged mix: k ~ U{1..kmax}, m = rs_from_str table[k], len ~ U[lmin..lmax]."""
    r = splitmix_words(seed, np.arange(g0, g0 + ng, dtype=np.uint64), 2)
    k = 1 + (r[:, 0] % np.uint64(kmax)).astype(np.int64)
    ln = lmin + (r[:, 1] % np.uint64(lmax - lmin + 1)).astype(np.int64)
    m = table_y[k - 1].astype(np.int64)
    return k, m, ln


HASH_SEED = 0xC4C4D16E57


def group_hashes(rows: np.ndarray) -> np.ndarray:
    """Per-group checksum of [G, R, L] uint8 rows (the checker's restatement of
    udpspeeder_amd.synth.group_hashes_dev): h_g = sum_j w_j * byte_j mod 2^64,
    w_j = mix(HASH_SEED + (j + 1) * GAMMA) | 1, j the byte's row-major index."""
    G = rows.shape[0]
    flat = np.ascontiguousarray(rows).reshape(G, -1)
    with np.errstate(over="ignore"):
        w = _mix(np.uint64(HASH_SEED) + np.arange(1, flat.shape[1] + 1, dtype=np.uint64) * GAMMA)
        w |= np.uint64(1)
        return flat.astype(np.uint64) @ w


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class _Lib:
    def __init__(self, path: str):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        self.lib = C.CDLL(path)


class Oracle(_Lib):
    """Our C restatement (librsoracle.so)."""

    def __init__(self, path: str = ORACLE_SO):
        super().__init__(path)
        L = self.lib
        L.orc_enc_matrix.argtypes = [C.c_int, C.c_int, C.c_void_p]
        L.orc_encode.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.orc_decode.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.orc_encode_batch.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64,
                                       C.c_int, C.c_int64]
        L.orc_decode_batch.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64,
                                       C.c_int, C.c_int64, C.c_void_p, C.c_void_p]
        L.orc_rs_from_str.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p]
        L.orc_gf_tables.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.orc_gf_mul.restype = C.c_uint8

    def gf_tables(self):
        e = np.zeros(510, np.uint8); lg = np.zeros(256, np.int32); inv = np.zeros(256, np.uint8)
        self.lib.orc_gf_tables(_p(e), _p(lg), _p(inv))
        return e, lg, inv

    def mul_table(self) -> np.ndarray:
        e, lg, _ = self.gf_tables()
        a = np.arange(256)
        t = e[(lg[:, None] + lg[None, :]) % 510]
        t[0, :] = 0
        t[:, 0] = 0
        return t.astype(np.uint8)

    def enc_matrix(self, k: int, n: int) -> np.ndarray:
        out = np.zeros((n, k), np.uint8)
        if self.lib.orc_enc_matrix(k, n, _p(out)) != 0:
            raise ValueError(f"invalid (k,n)=({k},{n})")
        return out

    def encode_batch(self, k, n, buf: np.ndarray, group_stride, shard_stride, length, ngroups):
        assert buf.flags.c_contiguous and buf.dtype == np.uint8
        assert (ngroups - 1) * group_stride + n * shard_stride <= buf.size or ngroups == 0
        rc = self.lib.orc_encode_batch(k, n, _p(buf), group_stride, shard_stride, length, ngroups)
        if rc:
            raise ValueError("orc_encode_batch failed")

    def decode_batch(self, k, n, buf, group_stride, shard_stride, length, ngroups, present):
        present = np.ascontiguousarray(present, dtype=np.uint8)
        assert present.shape == (ngroups, n)
        status = np.zeros(ngroups, np.int32)
        self.lib.orc_decode_batch(k, n, _p(buf), group_stride, shard_stride, length, ngroups,
                                  _p(present), _p(status))
        return status

    def rs_from_str(self, s: str):
        xs = np.zeros(256, np.uint8); ys = np.zeros(256, np.uint8)
        cnt = self.lib.orc_rs_from_str(s.encode(), _p(xs), _p(ys))
        if cnt < 0:
            return None
        return [(int(xs[i]), int(ys[i])) for i in range(cnt)]

    def decode_ptrs(self, k, n, shards: list, length):
        """Per-group rs_decode2 semantics on Python buffers: shards[i] is a
        bytearray or None.  Returns (rc, out) where out[i] is the index of the
        input buffer data[i] points to afterwards (or -1)."""
        bufs = [bytearray(s) + bytearray(max(0, 1 - len(s))) if s is not None else None
                for s in shards]
        keep = [(C.c_uint8 * max(length, 1)).from_buffer(b) if b is not None else None for b in bufs]
        arr = (C.c_void_p * n)(*[C.addressof(x) if x is not None else None for x in keep])
        addr = {C.addressof(x): i for i, x in enumerate(keep) if x is not None}
        rc = self.lib.orc_decode(k, n, arr, length)
        out = [addr.get(arr[i], -1) if arr[i] else -1 for i in range(n)]
        return rc, out, [bytes(b[:length]) if b is not None else None for b in bufs]


class Reference(_Lib):
    """The real reference codec (oracle/_ref/libref_rs.so), if it was built."""

    def __init__(self, path: str = REF_SO):
        super().__init__(path)
        L = self.lib
        L.ref_prewarm.argtypes = [C.c_int, C.c_int]
        L.ref_encode_batch.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64,
                                       C.c_int, C.c_int64, C.c_int]
        L.ref_decode_batch.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64,
                                       C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.ref_decode_ptrs.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int,
                                      C.c_void_p, C.c_void_p]

    @staticmethod
    def available(path: str = REF_SO) -> bool:
        return os.path.exists(path)

    def encode_batch(self, k, n, buf, group_stride, shard_stride, length, ngroups, nthreads=1):
        assert buf.flags.c_contiguous and buf.dtype == np.uint8
        rc = self.lib.ref_encode_batch(k, n, _p(buf), group_stride, shard_stride, length,
                                       ngroups, nthreads)
        if rc:
            raise ValueError("ref_encode_batch failed")

    def decode_batch(self, k, n, buf, group_stride, shard_stride, length, ngroups, present,
                     write_back=True, nthreads=1):
        present = np.ascontiguousarray(present, dtype=np.uint8)
        status = np.zeros(ngroups, np.int32)
        self.lib.ref_decode_batch(k, n, _p(buf), group_stride, shard_stride, length, ngroups,
                                  _p(present), _p(status), int(write_back), nthreads)
        return status

    def decode_ptrs(self, k, n, buf, shard_stride, length, in_slot):
        ins = np.ascontiguousarray(in_slot, dtype=np.int32)
        out = np.zeros(n, np.int32)
        rc = self.lib.ref_decode_ptrs(k, n, _p(buf), shard_stride, length, _p(ins), _p(out))
        return rc, out

    def enc_matrix(self, k: int, n: int) -> np.ndarray:
        """Recover fec_new's matrix through rs_encode2 alone: encoding unit
        vector e_j (1-byte shards) yields column j of the parity rows."""
        out = np.zeros((n, k), np.uint8)
        out[:k, :k] = np.eye(k, dtype=np.uint8)
        buf = np.zeros(n * k, np.uint8)  # group j = unit vector e_j
        for j in range(k):
            buf[j * n + j] = 1
        self.encode_batch(k, n, buf, n, 1, 1, k)
        out[k:, :] = buf.reshape(k, n)[:, k:].T
        return out


# --------------------------------------------------------------------------
# Packet cook / de_cook
# --------------------------------------------------------------------------
COOK_ORACLE_SO = os.path.join(HERE, "libcookoracle.so")
REF_COOK_SO = os.path.join(HERE, "_ref", "libref_cook.so")

NO_CHECKSUM, NO_OBSCURE, NO_XOR = 1, 2, 4
IV_MAX = 32          # packet.cpp:14 iv_max; the IV array stride of the batch API
COOK_SEED = 0xC00C1E5


def cook_payloads(seed: int, p0: int, npk: int, lens: np.ndarray, stride: int) -> np.ndarray:
    """[npk, stride] uint8: packet i's bytes 0..lens[i]-1 are SplitMix64 stream
    seed^(p0+i) (byte q = byte q%8 of word q//8), the rest zero."""
    lmax = int(lens.max()) if npk else 0
    words = splitmix_words(seed, np.arange(p0, p0 + npk, dtype=np.uint64), (lmax + 7) // 8)
    b = words.view(np.uint8).reshape(npk, -1)[:, :lmax]
    out = np.zeros((npk, stride), np.uint8)
    out[:, :lmax] = b
    out[np.arange(stride)[None, :] >= lens[:, None]] = 0
    return out


def cook_ivs(seed: int, p0: int, npk: int, iv_min: int = 4, iv_max: int = 32):
    """(iv [npk, 32] uint8, iv_len [npk] uint8): iv_len = random_between(iv_min,
    iv_max) as packet.cpp:81 draws it, bytes from a SplitMix64 stream."""
    r = splitmix_words(seed ^ 0x1F, np.arange(p0, p0 + npk, dtype=np.uint64), 5)
    iv_len = (iv_min + (r[:, 0] % np.uint64(iv_max - iv_min + 1))).astype(np.uint8)
    iv = np.ascontiguousarray(r[:, 1:5]).view(np.uint8).reshape(npk, 32).copy()
    return iv, iv_len


def device_ivs(seed: int, p0: int, npk: int):
    """The IVs rsmi_cook_dev draws when given none (cook.hip): words
    w_j = mix((seed ^ p) + (j+1)*GAMMA) of packet p; iv_len = 4 + w_0 % 29,
    iv byte j = byte j%8 of w_{1 + j//8}."""
    w = splitmix_words(seed, np.arange(p0, p0 + npk, dtype=np.uint64), 5)
    iv_len = (4 + (w[:, 0] % np.uint64(29))).astype(np.uint8)
    iv = np.ascontiguousarray(w[:, 1:5]).view(np.uint8).reshape(npk, 32).copy()
    return iv, iv_len


class CookOracle(_Lib):
    """Our C restatement of packet.cpp's cook (oracle/cook_oracle.c)."""

    def __init__(self, path: str = COOK_ORACLE_SO):
        super().__init__(path)
        L = self.lib
        L.co_crc32h.argtypes = [C.c_void_p, C.c_int]
        L.co_crc32h.restype = C.c_uint32
        L.co_do_cook.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_char_p, C.c_int]
        L.co_de_cook.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, C.c_int]
        L.co_cook_batch.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_char_p, C.c_int, C.c_void_p]
        L.co_decook_batch.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_char_p,
                                      C.c_int, C.c_void_p]

    def crc32h(self, data: bytes) -> int:
        b = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
        return int(self.lib.co_crc32h(_p(b), len(data)))

    def do_cook(self, data: bytes, iv: bytes, key: bytes = b"", flags: int = 0) -> bytes:
        buf = np.zeros(len(data) + 4 + len(iv) + 1 + 16, np.uint8)
        buf[:len(data)] = np.frombuffer(bytes(data), np.uint8)
        ivb = np.frombuffer(bytes(iv) + b"\0", np.uint8)
        n = self.lib.co_do_cook(_p(buf), len(data), _p(ivb), len(iv), key, flags)
        return buf[:n].tobytes()

    def de_cook(self, data: bytes, key: bytes = b"", flags: int = 0):
        """(status, bytes of the whole input buffer after the call, new len)."""
        buf = np.frombuffer(bytes(data) + b"\0", np.uint8).copy()
        ln = C.c_int(len(data))
        rc = self.lib.co_de_cook(_p(buf), C.byref(ln), key, flags)
        return rc, buf[:len(data)].tobytes(), ln.value

    def cook_batch(self, buf, stride, lens, iv, iv_len, key=b"", flags=0):
        npk = len(lens)
        lens = np.ascontiguousarray(lens, np.int32)
        out = np.zeros(npk, np.int32)
        self.lib.co_cook_batch(_p(buf), npk, stride, _p(lens), _p(np.ascontiguousarray(iv)),
                               _p(np.ascontiguousarray(iv_len, np.uint8)), key, flags, _p(out))
        return out

    def decook_batch(self, buf, stride, lens, key=b"", flags=0):
        npk = len(lens)
        lens = np.ascontiguousarray(lens, np.int32)
        out = np.zeros(npk, np.int32)
        self.lib.co_decook_batch(_p(buf), npk, stride, _p(lens), key, flags, _p(out))
        return out


class CookReference(_Lib):
    """The real reference packet.cpp (oracle/_ref/libref_cook.so), if built.
    Its transform state lives in process globals, so every call sets them."""

    def __init__(self, path: str = REF_COOK_SO):
        super().__init__(path)
        L = self.lib
        L.ref_cook_config.argtypes = [C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_int]
        L.ref_crc32h.argtypes = [C.c_void_p, C.c_int]
        L.ref_crc32h.restype = C.c_uint32
        L.ref_do_cook.argtypes = [C.c_void_p, C.c_int]
        L.ref_de_cook.argtypes = [C.c_void_p, C.c_void_p]
        L.ref_de_cook_batch.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                        C.c_int]
        L.ref_do_cook_batch.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]

    @staticmethod
    def available(path: str = REF_COOK_SO) -> bool:
        return os.path.exists(path)

    def config(self, key: bytes = b"", flags: int = 0, iv_min: int = 4, iv_max: int = 32):
        self.lib.ref_cook_config(flags & 1, (flags >> 1) & 1, (flags >> 2) & 1, key, iv_min, iv_max)

    def crc32h(self, data: bytes) -> int:
        b = np.frombuffer(bytes(data) + b"\0", np.uint8)
        return int(self.lib.ref_crc32h(_p(b), len(data)))

    def do_cook(self, data: bytes) -> bytes:
        buf = np.zeros(len(data) + 64, np.uint8)
        buf[:len(data)] = np.frombuffer(bytes(data), np.uint8)
        n = self.lib.ref_do_cook(_p(buf), len(data))
        return buf[:n].tobytes()

    def de_cook(self, data: bytes):
        buf = np.frombuffer(bytes(data) + b"\0", np.uint8).copy()
        ln = C.c_int(len(data))
        rc = self.lib.ref_de_cook(_p(buf), C.byref(ln))
        return rc, buf[:len(data)].tobytes(), ln.value

    def decook_batch(self, buf, stride, lens, nthreads=1):
        npk = len(lens)
        lens = np.ascontiguousarray(lens, np.int32)
        out = np.zeros(npk, np.int32)
        self.lib.ref_de_cook_batch(_p(buf), npk, stride, _p(lens), _p(out), nthreads)
        return out

    def cook_batch(self, buf, stride, lens):
        npk = len(lens)
        lens = np.ascontiguousarray(lens, np.int32)
        out = np.zeros(npk, np.int32)
        self.lib.ref_do_cook_batch(_p(buf), npk, stride, _p(lens), _p(out))
        return out


def recover_iv(cooked: bytes, plain_len: int, key: bytes = b"", flags: int = 0):
    """(iv, iv_len) a reference do_cook drew, read back from its output."""
    if flags & NO_OBSCURE:
        return b"", 0
    d = bytearray(cooked)
    if not (flags & NO_XOR) and key:
        for i in range(len(d)):
            d[i] ^= key[i % len(key)]
    ivl = d[-1]
    start = plain_len + (0 if flags & NO_CHECKSUM else 4)
    return bytes(d[start:start + ivl]), ivl
