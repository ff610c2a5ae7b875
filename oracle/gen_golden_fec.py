"""TEST INFRASTRUCTURE ONLY -- regenerate tests/golden/fec_encode.npz from the
REAL reference fec_encode_manager_t.

Run in the build container (where /root/reference exists):

    make -C oracle && python -m oracle.gen_golden_fec

Each case sets g_fec_par (-f string, mode, mtu, queue_len), feeds a fresh
reference manager a seeded event sequence -- packets of seeded lengths whose
bytes are the SplitMix64 stream of (seed, event index) (oracle.cpu.cook_payloads),
and input(0, 0) timer flushes -- and records every input() return value and
every packet output() returned, with the event it followed, unmodified: mode-0
groups carry the stale bytes of the reference's blob buffer past the blob's end
(blob_encode_t::output, fec_manager.cpp:67-75; the count of nonzero ones is
recorded), the managers being constructed in zeroed memory (ref_fec_driver.cpp).
The encoder's first sequence number (random in the reference) is read from its
first header.

Fixtures are data only: lengths, return codes, packet lengths / events, the
packet bytes themselves for the small cases and a sha256 of all of them.
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

from oracle.cpu import Reference, cook_payloads, splitmix_words
from oracle.fec_frame import EncodeManager, FecReference, lossy_channel, stale_bytes

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
FEC_SEED = 0xFEC0
FULL_BYTES_MAX = 120_000

# name, -f, mode, mtu, queue_len, events, max len, flush per mille, zero-len per mille
CASES = [
    ("m0_20_10", "20:10", 0, 1250, 200, 400, 1300, 20, 10),
    ("m0_c3", "1:3,2:4,10:6,20:10", 0, 1250, 200, 400, 400, 50, 20),
    ("m0_small_queue", "3:2", 0, 100, 5, 300, 60, 100, 50),
    ("m0_queue3", "20:10", 0, 1250, 3, 200, 500, 30, 0),
    ("m0_no_parity", "4:0", 0, 300, 200, 150, 200, 50, 50),
    ("m0_tiny", "2:1,8:4", 0, 40, 200, 300, 30, 60, 300),
    ("m1_20_10", "20:10", 1, 1250, 200, 300, 1200, 50, 10),
    ("m1_c3", "1:3,2:4,10:6,20:10", 1, 1250, 200, 400, 300, 100, 20),
    ("m1_no_parity", "5:0", 1, 1250, 200, 150, 100, 80, 50),
    ("m1_long", "3:2", 1, 1250, 200, 60, 3600, 100, 0),
]


def case_events(ci: int, n: int, lmax: int, flush_pm: int, zero_pm: int):
    r = splitmix_words(FEC_SEED ^ (ci << 20), np.arange(n, dtype=np.uint64), 3)
    lens = (r[:, 0] % np.uint64(lmax + 1)).astype(np.int64)
    lens[(r[:, 1] % np.uint64(1000)) < np.uint64(zero_pm)] = 0
    lens[(r[:, 2] % np.uint64(1000)) < np.uint64(flush_pm)] = -1
    lens = lens.astype(np.int32)
    pay = cook_payloads(FEC_SEED + ci, 0, n, np.maximum(lens, 0), max(1, int(lens.max(initial=0))))
    ev = [None if lens[i] < 0 else pay[i, :lens[i]].tobytes() for i in range(n)]
    return lens, ev


# Receive side (fec_decode_manager_t): the packets EncodeManager (pinned to the
# reference encoder above) frames for an encode case, seq0 fixed, through a
# seeded lossy channel, fed to the REAL reference decoder.
# name, encode case, seq0, channel kwargs
DEC_CASES = [
    ("d_m0_20_10", "m0_20_10", 0x10, dict(loss=0.15, dup=0.03, swap=0.1)),
    ("d_m0_c3", "m0_c3", 0xFFFFFFF8, dict(loss=0.3, dup=0.05, swap=0.2, replay=0.02)),
    ("d_m0_small_queue", "m0_small_queue", 7, dict(loss=0.2, swap=0.3, garbage=0.05)),
    ("d_m0_queue3", "m0_queue3", 99, dict(loss=0.25, dup=0.1, delay=0.02, delay_by=2100)),
    ("d_m0_tiny", "m0_tiny", 5, dict(loss=0.4, dup=0.1, swap=0.3, garbage=0.1)),
    ("d_m1_20_10", "m1_20_10", 0x20, dict(loss=0.15, dup=0.03, swap=0.1, trunc=0.02)),
    ("d_m1_c3", "m1_c3", 0xABCDEF, dict(loss=0.3, dup=0.05, swap=0.2, replay=0.03, trunc=0.03)),
    ("d_m1_no_parity", "m1_no_parity", 3, dict(loss=0.1, dup=0.1, garbage=0.05)),
    ("d_m1_long", "m1_long", 11, dict(loss=0.2, swap=0.2)),
]


def dec_channel(name: str):
    """The channel packets of a decode case (deterministic)."""
    ci = [c[0] for c in DEC_CASES].index(name)
    _, ename, seq0, kw = DEC_CASES[ci]
    ei = [c[0] for c in CASES].index(ename)
    _, rs, mode, mtu, ql, n, lmax, fpm, zpm = CASES[ei]
    lens, ev = case_events(ei, n, lmax, fpm, zpm)
    em = EncodeManager(rs, mode, mtu, ql, seq0)
    pk = []
    for e in ev:
        em.input(e)
        pk += em.output()
    return lossy_channel(pk, 0xC4A7 + ci, **kw)


def main():
    fr, rr = FecReference(), Reference()
    arrays = {}
    names = []
    for ci, (name, rs, mode, mtu, ql, n, lmax, fpm, zpm) in enumerate(CASES):
        fr.config(rs, mode, mtu, ql)
        lens, ev = case_events(ci, n, lmax, fpm, zpm)
        ret, pk, pev = fr.encode(ev)
        stale = 0
        if mode == 0:
            j = 0
            while j < len(pk):
                k, m = pk[j][5], pk[j][6]
                stale += stale_bytes(pk[j:j + k + m])
                j += k + m
        blob = b"".join(pk)
        seq0 = int.from_bytes(pk[0][:4], "big") if pk else 0
        arrays[f"{name}__lens"] = lens
        arrays[f"{name}__ret"] = np.asarray(ret, np.int32)
        arrays[f"{name}__pk_len"] = np.array([len(p) for p in pk], np.int32)
        arrays[f"{name}__pk_event"] = np.asarray(pev, np.int32)
        arrays[f"{name}__meta"] = np.array([ci, mode, mtu, ql, seq0, stale], np.int64)
        arrays[f"{name}__rs"] = np.frombuffer(rs.encode(), np.uint8)
        arrays[f"{name}__sha256"] = np.frombuffer(hashlib.sha256(blob).digest(), np.uint8)
        if len(blob) <= FULL_BYTES_MAX:
            arrays[f"{name}__pk_bytes"] = np.frombuffer(blob, np.uint8)
        names.append(name)
        print(f"{name}: {n} events, {len(pk)} packets, {len(blob)} B, nonzero stale bytes {stale}")
    arrays["cases"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "fec_encode.npz"), **arrays)

    arrays, names = {}, []
    for name, _, _, _ in DEC_CASES:
        chan = dec_channel(name)
        ret, out, oev = fr.decode(chan)
        blob = b"".join(out)
        arrays[f"{name}__chan_sha256"] = np.frombuffer(hashlib.sha256(b"".join(
            len(p).to_bytes(4, "little") + p for p in chan)).digest(), np.uint8)
        arrays[f"{name}__ret"] = np.asarray(ret, np.int32)
        arrays[f"{name}__out_len"] = np.array([len(p) for p in out], np.int32)
        arrays[f"{name}__out_event"] = np.asarray(oev, np.int32)
        arrays[f"{name}__sha256"] = np.frombuffer(hashlib.sha256(blob).digest(), np.uint8)
        if len(blob) <= FULL_BYTES_MAX:
            arrays[f"{name}__out_bytes"] = np.frombuffer(blob, np.uint8)
        names.append(name)
        rv = np.asarray(ret)
        print(f"{name}: {len(chan)} packets in, {len(out)} out ({len(blob)} B), "
              f"ret -1: {(rv == -1).sum()}, ret 0: {(rv == 0).sum()}")
    arrays["cases"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "fec_decode.npz"), **arrays)


if __name__ == "__main__":
    main()
