"""CPU: pin the cook/de_cook oracle (oracle/cook_oracle.c) against vectors made
by the reference's own packet.cpp (tests/golden/cook_vectors.npz), SURVEY §8f f2."""
import numpy as np
import pytest

from oracle.cpu import (NO_CHECKSUM, NO_OBSCURE, NO_XOR, CookReference, cook_ivs,
                        cook_payloads, recover_iv)


def test_crc32h_check_value(cook_oracle, cook_vectors):
    # packet.cpp:236-257 is the reflected CRC-32; the standard check value pins it.
    assert int(cook_vectors.z["crc_check"][0]) == 0xCBF43926
    assert cook_oracle.crc32h(b"123456789") == 0xCBF43926
    assert cook_oracle.crc32h(b"") == 0


def test_cook_matches_reference_vectors(cook_oracle, cook_vectors):
    for i in range(cook_vectors.n):
        c = cook_vectors.case(i)
        iv, ivl = recover_iv(c["cooked"], len(c["plain"]), c["key"], c["flags"])
        if not c["flags"] & NO_OBSCURE:
            assert 4 <= ivl <= 32                       # random_between(iv_min, iv_max)
        out = cook_oracle.do_cook(c["plain"], iv, c["key"], c["flags"])
        assert out == c["cooked"], i


def test_decook_matches_reference_vectors(cook_oracle, cook_vectors):
    for i in range(cook_vectors.n):
        c = cook_vectors.case(i)
        rc, buf, ln = cook_oracle.de_cook(c["cooked"], c["key"], c["flags"])
        assert rc == 0 and buf[:ln] == c["plain"], i


def test_decook_corrupted_matches_reference(cook_oracle, cook_vectors):
    seen = {0: 0, -1: 0}
    for i in range(cook_vectors.n):
        c = cook_vectors.case(i)
        if not c["bad_in"]:
            continue
        rc, buf, ln = cook_oracle.de_cook(c["bad_in"], c["key"], c["flags"])
        assert rc == c["bad_status"], i
        assert buf == c["bad_out"], i
        if rc == 0:
            assert ln == c["bad_len"]
        seen[rc] += 1
    assert seen[-1] > 50 and seen[0] > 0   # both outcomes exercised


def test_flag_lengths(cook_oracle):
    data = bytes(range(100))
    iv = bytes(range(7))
    assert len(cook_oracle.do_cook(data, iv)) == 100 + 4 + 7 + 1
    assert len(cook_oracle.do_cook(data, iv, flags=NO_CHECKSUM)) == 100 + 7 + 1
    assert len(cook_oracle.do_cook(data, iv, flags=NO_OBSCURE)) == 104
    assert cook_oracle.do_cook(data, iv, flags=NO_CHECKSUM | NO_OBSCURE | NO_XOR) == data
    # empty key: encrypt_0 is a no-op (packet.cpp:34)
    assert cook_oracle.do_cook(data, iv, b"", NO_CHECKSUM | NO_OBSCURE) == data


def test_decook_edge_cases(cook_oracle):
    assert cook_oracle.de_cook(b"", flags=0)[0] == -1                    # len < 1
    assert cook_oracle.de_cook(b"\x05", flags=NO_XOR)[0] == -1           # len < 1 + iv_len
    # iv_len 0 is a no-op de_obscure; then the crc must match
    body = b"hello"
    ck = cook_oracle.do_cook(body, b"", b"", NO_XOR)
    assert ck[-1] == 0
    rc, buf, ln = cook_oracle.de_cook(ck, b"", NO_XOR)
    assert rc == 0 and buf[:ln] == body
    assert cook_oracle.de_cook(b"\0\0\0", flags=NO_XOR | NO_OBSCURE)[0] == -1   # len - 4 < 0


def test_batch_matches_single(cook_oracle):
    npk, stride = 64, 1344
    lens = (np.arange(npk) * 37) % 1290
    buf = cook_payloads(0x1234, 0, npk, lens, stride)
    iv, ivl = cook_ivs(0x1234, 0, npk)
    want = [cook_oracle.do_cook(buf[i, :lens[i]].tobytes(), iv[i, :ivl[i]].tobytes(), b"key", 0)
            for i in range(npk)]
    out = cook_oracle.cook_batch(buf, stride, lens, iv, ivl, b"key", 0)
    for i in range(npk):
        assert buf[i, :out[i]].tobytes() == want[i]
    back = cook_oracle.decook_batch(buf, stride, out, b"key", 0)
    assert (back == lens).all()


@pytest.mark.skipif(not CookReference.available(), reason="reference not built here")
def test_random_against_live_reference(cook_oracle):
    ref = CookReference()
    rng = np.random.default_rng(7)
    for t in range(200):
        key = bytes(rng.integers(1, 256, rng.integers(0, 40)).astype(np.uint8))
        flags = int(rng.integers(0, 8))
        ref.config(key, flags)
        data = rng.integers(0, 256, int(rng.integers(0, 2000))).astype(np.uint8).tobytes()
        ck = ref.do_cook(data)
        iv, _ = recover_iv(ck, len(data), key, flags)
        assert cook_oracle.do_cook(data, iv, key, flags) == ck
        bad = bytearray(ck)
        if bad:
            bad[int(rng.integers(0, len(bad)))] ^= 0x10
        a, b = ref.de_cook(bytes(bad)), cook_oracle.de_cook(bytes(bad), key, flags)
        assert a[:2] == b[:2]
