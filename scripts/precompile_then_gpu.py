"""GPU box: warm the run-time network cache (rsmi_precompile_code) before any
GPU use, then initialise the GPU in the same process (tests/test_bitslice_rtc.py)."""
import os, sys, tempfile
sys.path.insert(0, os.getcwd())
os.environ.setdefault("RSMI_RTC_CACHE", tempfile.mkdtemp())
import udpspeeder_amd as u
from udpspeeder_amd._lib import check
print("code_encoder before", u.code_encoder(20, 30), flush=True)
u.precompile_code(10, 15)
print("precompiled", flush=True)
import torch
print("torch cuda", torch.cuda.is_available(), flush=True)
check(u.lib().rsmi_init(), "rsmi_init")
print("rsmi_init ok", flush=True)
