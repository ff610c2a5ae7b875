"""bench.py's measured HBM lines on their own: the copy variants and the
read:write mixes (rsmi_copy_peak), twice.  One JSON line each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import udpspeeder_amd as u
from udpspeeder_amd._lib import check

check(u.lib().rsmi_init(), "rsmi_init")
for _ in range(2):
    print(json.dumps(bench.hbm_copy_peak(u, torch, torch.device("cuda:0"))), flush=True)
