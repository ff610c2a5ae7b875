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
