"""CPU: the generated bit-sliced XOR networks (the code bitslice.hip inlines)
are bit-exact with the oracle for every specialised (k, n), and the
generator's matrix is fec_new's (golden fixtures from the reference)."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "udpspeeder_amd", "csrc")
INC = os.path.join(CSRC, "gen", "bitslice_codes.inc")
sys.path.insert(0, CSRC)
import gen_bitslice  # noqa: E402


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(INC):
        subprocess.run([sys.executable, os.path.join(CSRC, "gen_bitslice.py"), "--out", INC],
                       check=True)
    exe = str(tmp_path_factory.mktemp("bs") / "bitslice_host")
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "bitslice_host.cpp")], check=True)
    return exe


def codes():
    txt = open(INC).read() if os.path.exists(INC) else ""
    found = re.findall(r"X\((\d+), (\d+)\)", txt)
    return [(int(a), int(b)) for a, b in found] or gen_bitslice.default_codes()


def test_generator_matrix_is_fec_new(golden):
    for key in ["20_30", "10_16", "3_6", "1_4", "16_25", "7_13", "2_6", "4_8"]:
        k, n = map(int, key.split("_"))
        assert (np.array(gen_bitslice.enc_matrix(k, n), np.uint8) == golden.mats[key]).all()


def test_transpose_is_involution_and_transpose(harness):
    # covered implicitly by parity below; spot-check the generator's bit matrix
    for c in [1, 2, 0x53, 0xFF]:
        M = gen_bitslice.bitmat(c)
        for t in range(8):
            col = sum(M[u][t] << u for u in range(8))
            assert col == gen_bitslice.gmul(c, 1 << t)


@pytest.mark.parametrize("kn", gen_bitslice.default_codes())
def test_network_vs_oracle(harness, oracle, kn):
    k, n = kn
    m = n - k
    nchunks = 24
    rng = np.random.default_rng(k * 31 + n)
    data = rng.integers(0, 256, (nchunks, k, 32), dtype=np.uint8)
    data[0] = 0
    data[1] = 0xFF
    hdr = f"{k} {n} {nchunks}\n".encode()
    out = subprocess.run([harness], input=hdr + data.tobytes(), capture_output=True, check=True)
    par = np.frombuffer(out.stdout, np.uint8).reshape(nchunks, m, 32)
    ref = np.zeros((nchunks, n, 32), np.uint8)
    ref[:, :k] = data
    oracle.encode_batch(k, n, ref.reshape(-1), n * 32, 32, 32, nchunks)
    assert (par == ref[:, k:]).all()
