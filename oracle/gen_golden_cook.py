"""TEST INFRASTRUCTURE ONLY -- regenerate tests/golden/cook_vectors.npz from the
REAL reference packet transform.

Run in the build container (where /root/reference exists):

    make -C oracle && python -m oracle.gen_golden_cook

It drives oracle/_ref/libref_cook.so -- /root/reference/packet.cpp compiled
unmodified (with the reference sources it links against) by oracle/Makefile --
and records, for every (key, flags, length) case:

  plain      the packet handed to do_cook (SplitMix64 bytes, oracle/cpu.py)
  cooked     the reference do_cook output (its own mt19937 drew the IV; the IV is
             recoverable from the bytes, so these pin the transform exactly)
  bad        cooked with one bit flipped (or truncated), and the reference
             de_cook result on it: status, buffer after the call, and length

Fixtures are data only: concatenated byte arrays plus offset/length arrays.
crc32h's standard check value ("123456789" -> 0xCBF43926) is recorded too.
"""
from __future__ import annotations

import os

import numpy as np

from oracle.cpu import (COOK_SEED, CookReference, NO_CHECKSUM, NO_OBSCURE, NO_XOR,
                        splitmix_words)

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")

KEYS = [b"", b"k", b"passwd123", bytes(range(1, 200))]   # key_string is a C string (misc.cpp:628)
LENS = [0, 1, 3, 4, 5, 15, 16, 17, 33, 100, 1258]
BAD_MAX_LEN = 100


def _bytes(seed: int, idx: int, n: int) -> bytes:
    w = splitmix_words(seed, np.array([idx], np.uint64), (n + 7) // 8 + 1)
    return w.view(np.uint8)[:n].tobytes()


def main():
    ref = CookReference()
    cases = []  # (key_idx, flags, plain, cooked, bad_in, bad_status, bad_out, bad_len)
    i = 0
    for ki, key in enumerate(KEYS):
        for flags in range(8):
            ref.config(key, flags)
            for ln in LENS:
                plain = _bytes(COOK_SEED, i, ln)
                cooked = ref.do_cook(plain)
                rc, back, bl = ref.de_cook(cooked)
                assert rc == 0 and back[:bl] == plain, (ki, flags, ln)
                bad_in, bad_st, bad_out, bad_len = b"", 0, b"", 0
                if ln <= BAD_MAX_LEN and len(cooked):
                    r = splitmix_words(COOK_SEED ^ 0xBAD, np.array([i], np.uint64), 2)
                    c = bytearray(cooked)
                    if int(r[0, 0]) % 5 == 0:       # truncated packet
                        c = c[: int(r[0, 1]) % len(c)]
                    else:                           # one flipped bit
                        c[int(r[0, 1]) % len(c)] ^= 1 << (int(r[0, 0]) % 8)
                    bad_in = bytes(c)
                    bad_st, bad_out, bad_len = ref.de_cook(bad_in)
                cases.append((ki, flags, plain, cooked, bad_in, bad_st, bad_out, bad_len))
                i += 1

    def cat(col):
        parts = [c[col] for c in cases]
        off = np.cumsum([0] + [len(p) for p in parts]).astype(np.int64)
        return np.frombuffer(b"".join(parts) or b"\0", np.uint8)[: off[-1]].copy(), off

    plain, plain_off = cat(2)
    cooked, cooked_off = cat(3)
    bad_in, bad_off = cat(4)
    bad_out, _ = cat(6)
    keys = np.frombuffer(b"".join(k + b"\0" for k in KEYS), np.uint8)
    np.savez_compressed(
        os.path.join(OUT, "cook_vectors.npz"),
        keys=keys, key_idx=np.array([c[0] for c in cases], np.int32),
        flags=np.array([c[1] for c in cases], np.int32),
        plain=plain, plain_off=plain_off, cooked=cooked, cooked_off=cooked_off,
        bad_in=bad_in, bad_off=bad_off, bad_out=bad_out,
        bad_status=np.array([c[5] for c in cases], np.int32),
        bad_len=np.array([c[7] for c in cases], np.int32),
        crc_check=np.array([ref.crc32h(b"123456789")], np.uint32),
        flag_bits=np.array([NO_CHECKSUM, NO_OBSCURE, NO_XOR], np.int32))
    print(f"cook_vectors.npz: {len(cases)} cases, {plain.size + cooked.size + bad_in.size} bytes")


if __name__ == "__main__":
    main()
