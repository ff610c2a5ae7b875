"""Link-level drop-in: the reference's own
fec_manager.cpp, misc.cpp and companions, compiled unmodified WITHOUT
lib/fec.cpp and lib/rs.cpp and linked against librsmi.so
(oracle/_ref/libref_fec_rsmi.so, oracle/Makefile).  Its rs_encode2 /
rs_decode2 / fec_new / fec_free call sites (fec_manager.cpp:364, 632, 710;
misc.cpp:337-361) therefore run on the MI355X engine.  Test infrastructure
only: the product never loads anything under oracle/.

* the golden FEC encode / decode cases (generated from the all-reference
  build, tests/golden/fec_*.npz) replayed through it, byte for byte;
* the reference's own --unit-test (misc.cpp:305-540) through it, its
  transcript against the all-reference build's.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle.fec_frame import REF_FEC_SO, FecReference
from oracle.gen_golden_fec import CASES, DEC_CASES, case_events, dec_channel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_FEC_RSMI_SO = os.path.join(ROOT, "oracle", "_ref", "libref_fec_rsmi.so")

need_link = pytest.mark.skipif(not os.path.exists(REF_FEC_RSMI_SO),
                               reason="oracle/_ref/libref_fec_rsmi.so not built")


def test_link_has_no_reference_codec():
    """The linked build holds none of lib/fec.cpp's or lib/rs.cpp's code: its
    rs_* / fec_* symbols are undefined there and bound to librsmi.so."""
    if not os.path.exists(REF_FEC_RSMI_SO):
        pytest.skip("oracle/_ref/libref_fec_rsmi.so not built")
    out = subprocess.run(["nm", "-D", REF_FEC_RSMI_SO], capture_output=True, text=True).stdout
    syms = {l.split()[-1]: l.split()[-2] for l in out.splitlines() if l.strip()}
    for s in ["_Z10rs_encode2iiPPci", "_Z10rs_decode2iiPPci", "_Z7fec_newii", "_Z8fec_freePv"]:
        assert syms.get(s) == "U", s
    for s in syms:
        assert "invert_mat" not in s and "addmul" not in s and "generate_gf" not in s
    needed = subprocess.run(["readelf", "-d", REF_FEC_RSMI_SO], capture_output=True,
                            text=True).stdout
    assert "[librsmi.so]" in needed


@pytest.mark.gpu
@need_link
@pytest.mark.parametrize("name", [c[0] for c in CASES])
def test_reference_encode_manager_on_dropin(gpu, name):
    fx = dict(np.load(os.path.join(GOLDEN, "fec_encode.npz")))
    ci = [c[0] for c in CASES].index(name)
    _, rs, mode, mtu, ql, n, lmax, fpm, zpm = CASES[ci]
    _, ev = case_events(ci, n, lmax, fpm, zpm)
    fr = FecReference(REF_FEC_RSMI_SO)
    fr.config(rs, mode, mtu, ql)
    ret, pk, pev = fr.encode(ev)
    assert list(ret) == list(fx[f"{name}__ret"])
    assert list(pev) == list(fx[f"{name}__pk_event"])
    assert [len(p) for p in pk] == list(fx[f"{name}__pk_len"])
    # the first sequence number is random in the reference: compare the rest
    seq0 = int(fx[f"{name}__meta"][4])
    got0 = int.from_bytes(pk[0][:4], "big") if pk else seq0
    fixed = [((int.from_bytes(p[:4], "big") - got0 + seq0) & 0xFFFFFFFF).to_bytes(4, "big") + p[4:]
             for p in pk]
    assert hashlib.sha256(b"".join(fixed)).digest() == fx[f"{name}__sha256"].tobytes()


@pytest.mark.gpu
@need_link
@pytest.mark.parametrize("name", [c[0] for c in DEC_CASES])
def test_reference_decode_manager_on_dropin(gpu, name):
    fx = dict(np.load(os.path.join(GOLDEN, "fec_decode.npz")))
    chan = dec_channel(name)
    fr = FecReference(REF_FEC_RSMI_SO)
    ret, out, oev = fr.decode(chan)
    assert list(ret) == list(fx[f"{name}__ret"])
    assert list(oev) == list(fx[f"{name}__out_event"])
    assert [len(p) for p in out] == list(fx[f"{name}__out_len"])
    assert hashlib.sha256(b"".join(out)).digest() == fx[f"{name}__sha256"].tobytes()


# process_arg leaves g_fec_par at its defaults before --unit-test runs
# (misc.cpp:587-594): -f 20:10, mode 0, mtu 1250, queue 200
_UNIT = ("import ctypes, sys; lib = ctypes.CDLL(sys.argv[1]); "
         "lib.ref_fec_config(b'20:10', 0, 1250, 200); sys.stdout.flush(); lib._Z9unit_testv()")


def _unit_transcript(so):
    p = subprocess.run([sys.executable, "-c", _UNIT, so], capture_output=True, timeout=120,
                       cwd=ROOT)  # bytes: the transcript prints parity shards with %s
    assert p.returncode == 0, p.stderr[-2000:]
    lines = p.stdout.split(b"\n")
    return lines[2:]  # the first two lines print get_fake_random_chars (random)


@pytest.mark.gpu
@need_link
def test_reference_unit_test_on_dropin(gpu):
    """misc.cpp's --unit-test (RS(3,6) KAT through rs_encode2/rs_decode2, blob
    round trip, mode-0 manager round trips) on the drop-in: same transcript as
    the all-reference build."""
    if not os.path.exists(REF_FEC_SO):
        pytest.skip("reference FEC build absent")
    want = _unit_transcript(REF_FEC_SO)
    got = _unit_transcript(REF_FEC_RSMI_SO)
    assert got == want
    assert any(b"<aaa><bbb><ccc>" in l for l in got)
