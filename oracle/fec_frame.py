"""TEST INFRASTRUCTURE ONLY -- a CPU restatement of UDPspeeder's FEC framing
(SURVEY §8f row f1), the checker for include/rsmi_fec.h.  Nothing here is
shipped or called by the product path.

* :class:`EncodeManager` restates ``fec_encode_manager_t::input`` / ``output``
  (fec_manager.cpp:174-460) and ``blob_encode_t`` (:35-75) in plain Python;
  parity comes from the C restatement of lib/fec.cpp (oracle/rs_oracle.c).
  One deliberate difference from the reference, the same as the GPU path's:
  in mode 0 the bytes of the last data shard past the blob's end are zero,
  where the reference sends stale bytes of earlier blobs.
* :class:`FecReference` drives the REAL reference managers
  (oracle/_ref/libref_fec.so, fec_manager.cpp compiled unmodified), for the
  golden generator and for pinning this restatement.
* :func:`stale_bytes` counts the stale blob-buffer bytes a mode-0 group
  carries past its blob (reproduced by the restatement and the GPU path).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Tuple

import numpy as np

from oracle.cpu import Oracle

HERE = os.path.dirname(os.path.abspath(__file__))
REF_FEC_SO = os.path.join(HERE, "_ref", "libref_fec.so")
HEADER = 8
MAX_FEC_PACKET_NUM = 255


def rs_table(rs_str: str) -> List[int]:
    """rs_par[x-1].y for x = 1..rs_cnt (fec_manager.h:40-136)."""
    from udpspeeder_amd.fec_param import rs_from_str
    t = rs_from_str(rs_str)
    if t is None:
        raise ValueError(rs_str)
    return [y for _, y in t]


def _round_up_div(a: int, b: int) -> int:  # common.cpp:747-749
    return (a + b - 1) // b


def _hdr(seq: int, mode: int, k: int, m: int, idx: int) -> bytes:  # fec_manager.cpp:318-333
    return seq.to_bytes(4, "big") + bytes([mode, k, m, idx & 0xFF])


class EncodeManager:
    """fec_encode_manager_t restated.  input(None) is input(0, 0)."""

    def __init__(self, rs_str: str, mode: int, mtu: int, queue_len: int, seq0: int,
                 short_packet_optimize: int = 1, header_overhead: int = 40,
                 oracle: Optional[Oracle] = None):
        self.y = rs_table(rs_str)
        self.mode, self.mtu, self.queue_len = mode, mtu, queue_len
        self.spo, self.overhead = short_packet_optimize, header_overhead
        self.seq = seq0 & 0xFFFFFFFF
        self.pend: List[bytes] = []
        self.blob_len = 4
        # blob_encode_t::input_buf (fec_manager.h:257): never cleared, so the
        # bytes past a blob's end are what earlier, longer blobs left there
        # (blob_encode_t::output, fec_manager.cpp:67-75); zero at first
        self.blob_buf = bytearray()
        self.ready: List[bytes] = []
        self.oracle = oracle or Oracle()

    @property
    def tail_x(self) -> int:
        return len(self.y)

    def _shard_len(self, n: int, nxt: int) -> int:  # blob_encode_t::get_shard_len :51-53
        return _round_up_div(self.blob_len + 2 + nxt, n)

    def _append(self, s: bytes):  # :174-204
        self.pend.append(bytes(s))
        if self.mode == 0:
            self.blob_len += 2 + len(s)

    def _parity(self, shards: List[bytes], k: int, n: int, ln: int) -> List[bytes]:
        stride = max(16, (ln + 15) // 16 * 16)
        buf = np.zeros(n * stride, np.uint8)
        for i, s in enumerate(shards):
            buf[i * stride:i * stride + ln] = np.frombuffer(s, np.uint8)
        self.oracle.encode_batch(k, n, buf, n * stride, stride, ln, 1)
        return [buf[j * stride:j * stride + ln].tobytes() for j in range(k, n)]

    def input(self, s: Optional[bytes]) -> int:
        mode = self.mode
        has = s is not None
        ln = len(s) if has else 0
        if has and ln > 65535:
            return -1
        if mode == 0 and has and not self.pend:
            if self._shard_len(self.tail_x, ln) > self.mtu:  # :217-223
                return -1
        if not has and not self.pend:  # :228-231
            return -1
        about = not has
        delayed = False
        if mode == 0 and self._shard_len(self.tail_x, ln) > self.mtu:  # :235-238
            about = delayed = True
        if has and not delayed:
            self._append(s)
        counter = len(self.pend)
        if mode == 0 and counter == self.queue_len:
            about = True
        if mode == 1 and counter == self.tail_x:
            about = True
        out: List[bytes] = []
        if about:
            if mode == 0:
                tx = self.tail_x
                k, m = tx, self.y[tx - 1]
                if self.spo:  # short_packet_optimize :264-288
                    best_len = (self._shard_len(tx, 0) + self.overhead) * (tx + m)
                    best = tx
                    for i in range(1, tx):
                        sl = self._shard_len(i, 0)
                        if sl > self.mtu:
                            continue
                        nl = (sl + self.overhead) * (i + self.y[i - 1])
                        if nl < best_len:
                            best_len, best = nl, i
                    k, m = best, self.y[best - 1]
                fec_len = _round_up_div(self.blob_len, k)
                blob = bytearray(len(self.pend).to_bytes(4, "big"))
                for p in self.pend:
                    blob += len(p).to_bytes(2, "big") + p
                cl = len(blob)
                tail = bytes(self.blob_buf[cl:k * fec_len])
                blob += tail + bytes(k * fec_len - cl - len(tail))  # stale bytes, as sent
                if len(self.blob_buf) < cl:
                    self.blob_buf += bytes(cl - len(self.blob_buf))
                self.blob_buf[:cl] = blob[:cl]
                data = [bytes(blob[i * fec_len:(i + 1) * fec_len]) for i in range(k)]
                par = self._parity(data, k, k + m, fec_len)
                for i in range(k + m):
                    out.append(_hdr(self.seq, 0, k, m, i) + (data + par)[i])
            else:
                k = counter
                m = self.y[counter - 1]
                fec_len = max(len(p) + 2 for p in self.pend)
                data = [(len(p).to_bytes(2, "big") + p).ljust(fec_len, b"\0") for p in self.pend]
                par = self._parity(data, k, k + m, fec_len)
                if has:  # fast send: the last data packet goes with the parity
                    out.append(_hdr(self.seq, 1, 0, 0, k - 1) + data[k - 1][:len(self.pend[-1]) + 2])
                for i in range(k, k + m):
                    out.append(_hdr(self.seq, 1, k, m, i) + par[i - k])
            self.seq = (self.seq + 1) & 0xFFFFFFFF
            self.pend = []
            self.blob_len = 4
        elif has and mode == 1:  # encode_fast_send :394-429
            i = counter - 1
            out.append(_hdr(self.seq, 1, 0, 0, i) + len(s).to_bytes(2, "big") + bytes(s))
        if has and delayed:
            self._append(s)
        self.ready = out
        return 0

    def output(self) -> List[bytes]:
        r, self.ready = self.ready, []
        return r


def stale_bytes(packets: List[bytes]) -> int:
    """Nonzero bytes past the blob's end in a mode-0 group (all k+m packets):
    the stale content of blob_encode_t's buffer the reference sends."""
    k = packets[0][5]
    blob = b"".join(p[HEADER:] for p in packets[:k])
    cnt = int.from_bytes(blob[:4], "big")
    pos = 4
    for _ in range(cnt):
        pos += 2 + int.from_bytes(blob[pos:pos + 2], "big")
    return sum(1 for b in blob[pos:] if b)


class FecReference:
    """The real reference managers (oracle/_ref/libref_fec.so).  The managers'
    parameters live in the process-global g_fec_par; config() sets them and
    managers created afterwards copy them (fec_manager.cpp:154)."""

    def __init__(self, path: str = REF_FEC_SO):
        self.lib = C.CDLL(path)
        L = self.lib
        L.ref_fec_config.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int]
        L.ref_fenc_new.restype = C.c_void_p
        L.ref_fenc_free.argtypes = [C.c_void_p]
        L.ref_fdec_new.restype = C.c_void_p
        L.ref_fdec_free.argtypes = [C.c_void_p]
        for f in (L.ref_fenc_run, L.ref_fdec_run):
            f.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                          C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
            f.restype = C.c_int64

    @staticmethod
    def available(path: str = REF_FEC_SO) -> bool:
        return os.path.exists(path)

    def config(self, rs_str: str, mode: int, mtu: int = 1250, queue_len: int = 200):
        if self.lib.ref_fec_config(rs_str.encode(), mode, mtu, queue_len) != 0:
            raise ValueError(rs_str)

    def _run(self, fn, h, events: List[Optional[bytes]]):
        n = len(events)
        lens = np.array([-1 if e is None else len(e) for e in events], np.int32)
        offs = np.zeros(n, np.uint64)
        o = 0
        for i, e in enumerate(events):
            offs[i] = o
            o += 0 if e is None else len(e)
        buf = np.frombuffer(b"".join(e for e in events if e is not None) + bytes(16), np.uint8).copy()
        ret = np.zeros(n, np.int32)
        cap = max(1 << 20, 64 * (o + 1) + 4096 * n)
        maxo = 300 * n + 16
        out = np.zeros(cap, np.uint8)
        pos = np.zeros(maxo, np.int64)
        ol = np.zeros(maxo, np.int32)
        ev = np.zeros(maxo, np.int32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        np_ = fn(h, n, p(lens), p(offs), p(buf), p(ret), p(out), cap, p(pos), p(ol), p(ev), maxo)
        if np_ < 0:
            raise RuntimeError("reference output overflow")
        pk = [out[pos[j]:pos[j] + ol[j]].tobytes() for j in range(np_)]
        return ret, pk, ev[:np_].copy()

    def encode(self, events: List[Optional[bytes]]):
        """Feed a fresh fec_encode_manager_t; returns (ret[], packets[], event[])."""
        h = self.lib.ref_fenc_new()
        try:
            return self._run(self.lib.ref_fenc_run, h, events)
        finally:
            self.lib.ref_fenc_free(h)

    def decode(self, packets: List[bytes]):
        """Feed a fresh fec_decode_manager_t; returns (ret[], outputs[], event[])."""
        h = self.lib.ref_fdec_new()
        try:
            return self._run(self.lib.ref_fdec_run, h, packets)
        finally:
            self.lib.ref_fdec_free(h)


# --------------------------------------------------------------------------
# fec_decode_manager_t (fec_manager.cpp:469-797, fec_manager.h:185-235, 366-435)
FEC_BUFF_NUM = 2000              # fec_manager.cpp:33
ANTI_REPLAY_BUFF_SIZE = 30000    # fec_manager.h:16
ANTI_REPLAY_TIMEOUT = 120 * 1000  # fec_manager.h:185 (ms)
MAX_DATA_LEN = 3600              # common.h:102


class AntiReplay:
    """anti_replay_t (fec_manager.h:187-235); time in ms from the caller."""

    def __init__(self):
        self.buf = [-1] * ANTI_REPLAY_BUFF_SIZE
        self.mp = {}  # seq -> [time, index]
        self.index = 0

    def is_valid(self, seq: int, now: int) -> bool:
        e = self.mp.get(seq)
        if e is None:
            return True
        if now - e[0] > ANTI_REPLAY_TIMEOUT:
            self.buf[e[1]] = -1
            del self.mp[seq]
            return True
        return False

    def set_invalid(self, seq: int, now: int):
        if not self.is_valid(seq, now):
            return
        old = self.buf[self.index]
        if old != -1:
            del self.mp[old]
        self.buf[self.index] = seq
        self.mp[seq] = [now, self.index]
        self.index = (self.index + 1) % ANTI_REPLAY_BUFF_SIZE


class _Group:  # fec_group_t (fec_manager.h:376-384)
    __slots__ = ("type", "data_num", "redundant_num", "len", "fec_done", "group_mp")

    def __init__(self):
        self.type = self.data_num = self.redundant_num = self.len = -1
        self.fec_done = 0
        self.group_mp = {}  # inner index -> ring slot


class DecodeManager:
    """fec_decode_manager_t restated; parity via the C restatement of
    rs_decode2.  input(packet) -> return value; output() -> list of bytes."""

    def __init__(self, oracle: Optional[Oracle] = None):
        self.oracle = oracle or Oracle()
        self.ar = AntiReplay()
        self.mp = {}
        self.ring = [None] * FEC_BUFF_NUM  # (seq, payload bytes) per slot
        self.index = 0
        self.ready: List[bytes] = []
        self.now = 0  # ms

    def _g(self, seq) -> _Group:  # unordered_map::operator[] inserts
        g = self.mp.get(seq)
        if g is None:
            g = self.mp[seq] = _Group()
        return g

    def input(self, s: bytes) -> int:
        self.ready = []
        r = self._input(bytes(s))
        return r

    def _input(self, s: bytes) -> int:
        if len(s) < HEADER:
            return -1
        seq = int.from_bytes(s[:4], "big")
        typ, data_num, red_num, inner = s[4], s[5], s[6], s[7]
        pay = s[HEADER:]
        ln = len(pay)
        if typ == 1:
            if ln < 2:
                return -1
            if data_num == 0 and int.from_bytes(pay[:2], "big") + 2 != ln:
                return -1
        if typ == 0 and data_num == 0:
            return -1
        if data_num + red_num >= MAX_FEC_PACKET_NUM:
            return -1
        if not self.ar.is_valid(seq, self.now):
            return 0
        g = self._g(seq)
        if g.fec_done:
            return -1
        if inner in g.group_mp:
            return -1
        if g.type == -1:
            g.type = typ
        elif g.type != typ:
            return -1
        if data_num != 0:
            if g.data_num == -1:
                g.data_num, g.redundant_num, g.len = data_num, red_num, ln
            elif (g.data_num, g.redundant_num, g.len) != (data_num, red_num, ln):
                return -1
        old = self.ring[self.index]
        if old is not None:
            tmp_seq = old[0]
            self.ar.set_invalid(tmp_seq, self.now)
            self.mp.pop(tmp_seq, None)
            if tmp_seq == seq:
                return -1
        self.ring[self.index] = (seq, pay)
        g = self._g(seq)
        g.group_mp[inner] = self.index
        size = len(g.group_mp)
        about = False
        end = False
        if typ == 0:
            if size > data_num:
                self.ar.set_invalid(seq, self.now)
                end = True
            elif size == data_num:
                about = True
        elif g.data_num != -1:
            if size > g.data_num + 1:
                self.ar.set_invalid(seq, self.now)
                end = True
            elif size >= g.data_num:
                about = True
        if not end:
            if about:
                self._decode(seq, g, typ, inner, ln)
            elif typ == 1 and data_num == 0:  # decode_fast_send (:760-776)
                self.ready = [pay[2:]]
        self.index = (self.index + 1) % FEC_BUFF_NUM
        return 0

    def _decode(self, seq, g: _Group, typ, inner, ln):
        k, m = g.data_num, g.redundant_num
        n = k + m
        if typ == 0:
            shards = [None] * n
            for idx, slot in g.group_mp.items():
                if idx < n:
                    shards[idx] = self.ring[slot][1]
            bad_index = any(idx >= n for idx in g.group_mp)
            rc, out, bufs = self.oracle.decode_ptrs(k, n, shards, ln) if not bad_index else (1, None, None)
            g.fec_done = 1
            if rc != 0:  # the reference asserts here (fec_manager.cpp:632)
                self.ar.set_invalid(seq, self.now)
                return
            blob = b"".join(bufs[out[i]] for i in range(k))
            if len(blob) < 4:
                self.ar.set_invalid(seq, self.now)
                return
            cnt = int.from_bytes(blob[:4], "big")
            if cnt > 30000:  # max_blob_packet_num (fec_manager.h:15)
                self.ar.set_invalid(seq, self.now)
                return
            pos, res = 4, []
            for _ in range(cnt):  # blob_decode_t::output (:97-129)
                if pos + 2 > len(blob):
                    self.ar.set_invalid(seq, self.now)
                    return
                l = int.from_bytes(blob[pos:pos + 2], "big")
                pos += 2
                if pos + l > len(blob):
                    self.ar.set_invalid(seq, self.now)
                    return
                res.append(blob[pos:pos + l])
                pos += l
            self.ready = res
            self.ar.set_invalid(seq, self.now)
        else:
            items = sorted(g.group_mp.items())
            lens = [len(self.ring[slot][1]) for _, slot in items]
            max_len = max(lens)
            if min(lens) < 2 or max_len != g.len:
                self.ar.set_invalid(seq, self.now)
                return
            shards = [None] * n
            for idx, slot in items:
                if idx < n:
                    shards[idx] = self.ring[slot][1].ljust(max_len, b"\0")
            missed = [i for i in range(k) if shards[i] is None or i == inner]
            bad_index = any(idx >= n for idx, _ in items)
            rc, out, bufs = self.oracle.decode_ptrs(k, n, shards, max_len) if not bad_index else (1, None, None)
            g.fec_done = 1
            if rc != 0:  # the reference asserts here (fec_manager.cpp:710)
                self.ar.set_invalid(seq, self.now)
                return
            data = [bufs[out[i]] for i in range(k)]
            lens_i = [int.from_bytes(d[:2], "big") for d in data]
            if all(l <= MAX_DATA_LEN for l in lens_i):
                # a malformed row can claim more bytes than it holds: the reference
                # then reads past the row into stale ring-buffer memory
                # (fec_manager.cpp:715-717); here those bytes are zero (documented)
                self.ready = [data[i][2:2 + lens_i[i]].ljust(lens_i[i], b"\0") for i in missed]
            self.ar.set_invalid(seq, self.now)

    def output(self) -> List[bytes]:
        r, self.ready = self.ready, []
        return r


def lossy_channel(packets: List[bytes], seed: int, loss=0.1, dup=0.02, swap=0.05, delay=0.0,
                  delay_by=2500, replay=0.0, trunc=0.0, garbage=0.0) -> List[bytes]:
    """A seeded unreliable channel for decode tests: drops, duplicates, swaps
    neighbours, delays packets by ~delay_by positions (past the reference's
    2000-buffer ring), replays old packets (anti-replay), truncates mode-1
    packets by 1..3 bytes and injects short / out-of-range garbage headers.
    Deterministic in (packets, seed)."""
    rng = np.random.default_rng(seed)
    out: List[bytes] = []
    held: List[Tuple[int, bytes]] = []
    for p in packets:
        while held and held[0][0] <= len(out):
            out.append(held.pop(0)[1])
        r = rng.random(8)
        if r[0] < loss:
            continue
        q = p
        if r[1] < trunc and len(q) > HEADER + 3 and q[4] == 1:
            q = q[:len(q) - 1 - int(rng.integers(0, 3))]
        if r[2] < delay:
            held.append((len(out) + delay_by + int(rng.integers(0, 500)), q))
            held.sort(key=lambda t: t[0])
        else:
            out.append(q)
        if r[3] < dup:
            out.append(q)
        if r[4] < replay and len(out) > 50:
            out.append(out[int(rng.integers(0, len(out) - 50))])
        if r[5] < garbage:
            kind = int(rng.integers(0, 3))
            if kind == 0:
                out.append(bytes(rng.integers(0, 256, int(rng.integers(0, 8)), dtype=np.uint8)))
            elif kind == 1:  # data_num + redundant_num >= 255
                out.append(q[:5] + bytes([200, 60]) + q[7:])
            else:  # type 0 with data_num 0
                out.append(q[:4] + bytes([0, 0]) + q[6:])
    out += [p for _, p in held]
    for i in range(len(out) - 1):
        if rng.random() < swap:
            out[i], out[i + 1] = out[i + 1], out[i]
    return out
