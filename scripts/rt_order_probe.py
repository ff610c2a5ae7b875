"""GPU box: which first-use order of librsmi / hipRTC / torch leaves the HIP
runtime with its devices (diagnostic for rsmi_precompile_code before GPU use).
Usage: python scripts/rt_order_probe.py <variant>"""
import os, sys, tempfile
sys.path.insert(0, os.getcwd())
os.environ.setdefault("RSMI_RTC_CACHE", tempfile.mkdtemp())
v = sys.argv[1]
if v in ("torch_first", "torch_first_cuda"):
    import torch
    if v == "torch_first_cuda":
        print("cuda", torch.cuda.is_available(), flush=True)
import udpspeeder_amd as u
u.lib()
if v != "no_rtc":
    u.precompile_code(10, 15)
import torch
print(v, "cuda", torch.cuda.is_available(), flush=True)
rc = u.lib().rsmi_init()
print(v, "rsmi_init", rc, u.lib().rsmi_last_error().decode() if rc else "ok", flush=True)
