import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle.cpu import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    class G:
        kat = json.load(open(os.path.join(GOLDEN, "kat_rs3_6.json")))
        full = json.load(open(os.path.join(GOLDEN, "full_hashes.json")))
        mats = dict(np.load(os.path.join(GOLDEN, "matrices.npz")))
        enc = dict(np.load(os.path.join(GOLDEN, "encode_small.npz")))
        dec = dict(np.load(os.path.join(GOLDEN, "decode_small.npz")))
    return G


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import udpspeeder_amd as u
    from udpspeeder_amd._lib import check
    check(u.lib().rsmi_init(), "rsmi_init")
    return torch.device("cuda:0")


class CookVectors:
    """tests/golden/cook_vectors.npz (made by oracle/gen_golden_cook.py from the
    real packet.cpp): per-case key, flags, plain/cooked bytes and a corrupted
    de_cook case."""

    def __init__(self, path=os.path.join(GOLDEN, "cook_vectors.npz")):
        z = dict(np.load(path))
        self.z = z
        self.keys = z["keys"].tobytes().split(b"\0")[:-1]
        self.n = len(z["flags"])

    def _cut(self, arr, off, i):
        return self.z[arr][self.z[off][i]:self.z[off][i + 1]].tobytes()

    def case(self, i):
        z = self.z
        return dict(key=self.keys[z["key_idx"][i]], flags=int(z["flags"][i]),
                    plain=self._cut("plain", "plain_off", i),
                    cooked=self._cut("cooked", "cooked_off", i),
                    bad_in=self._cut("bad_in", "bad_off", i),
                    bad_out=self._cut("bad_out", "bad_off", i),
                    bad_status=int(z["bad_status"][i]), bad_len=int(z["bad_len"][i]))


@pytest.fixture(scope="session")
def cook_vectors():
    return CookVectors()


@pytest.fixture(scope="session")
def cook_oracle():
    from oracle.cpu import CookOracle
    return CookOracle()
