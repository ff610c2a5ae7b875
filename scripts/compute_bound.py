"""Measurement: the encode / decode kernels with every group aliased onto one
group's slots (group_stride 0), so loads hit in cache and the kernel time is
its instruction cost; beside the normal HBM-streaming time.  Library from
RSMI_LIB."""
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import udpspeeder_amd as u  # noqa: E402
from udpspeeder_amd import synth  # noqa: E402
from udpspeeder_amd._lib import check, lib  # noqa: E402

k, n, ln, G, S = 20, 30, 1250, 65536, 1280


def timed(fn, reps=30):
    ts = []
    for i in range(reps + 5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        if i >= 5:
            ts.append(a.elapsed_time(b))
    return statistics.median(ts)


one = torch.zeros((4, n, S), dtype=torch.uint8, device="cuda")
u.fill_data(one, k, ln, 3)
full = torch.zeros((G, n, S), dtype=torch.uint8, device="cuda")
u.fill_data(full, k, ln, 3)
pres = torch.from_numpy(synth.erasure_present(synth.ERASE_SEED, 0, G, n, 5)).cuda()
st = torch.empty(G, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
L = lib()
enc_alias = timed(lambda: check(L.rsmi_encode_dev(k, n, one.data_ptr(), 0, S, ln, G, s), "enc"))
dec_alias = timed(lambda: check(L.rsmi_decode_dev(k, n, one.data_ptr(), 0, S, ln, G, pres.data_ptr(),
                                                  st.data_ptr(), s), "dec"))
u.encode(full, k, n, ln)
enc = timed(lambda: u.encode(full, k, n, ln))
dec = timed(lambda: u.decode(full, pres, k, n, ln, status=st))
name = os.path.basename(os.environ.get("RSMI_LIB", "default"))
print(f"{name}: encode aliased {enc_alias:.4f} ms, streaming {enc:.4f} ms | "
      f"decode aliased {dec_alias:.4f} ms, streaming {dec:.4f} ms", flush=True)
