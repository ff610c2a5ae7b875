"""Bit-sliced encoders for codes without a build-time network (SURVEY §8 row
a6 for every code rs_from_str admits, fec_manager.h:40-136; matrix of fec_new,
lib/fec.cpp:665-720): librsmi emits the XOR network in C++ and compiles it
with hipRTC (udpspeeder_amd/csrc/bitslice_rtc.cpp).

CPU: the C++ emitter prints exactly the build-time generator's text; the
emitted networks (incl. multi-pass ones, > 10 parity rows) run in the host
harness bit-exact with the oracle; hipRTC compiles them without a GPU.
GPU: uniform and ragged encodes through the run-time kernels against the
oracle."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "udpspeeder_amd", "csrc")
sys.path.insert(0, CSRC)
import gen_bitslice  # noqa: E402

# not in the build-time set; (10,40), (5,17), (30,42), (2,200) take several passes
RTC_CODES = [(10, 15), (1, 2), (3, 4), (10, 40), (5, 17), (30, 42), (7, 9), (2, 200), (40, 60)]


@pytest.fixture(scope="module")
def u(tmp_path_factory):
    """This module's compiles go to a private cache; the variable is restored
    afterwards, so later modules keep the default (warm) cache."""
    old = os.environ.get("RSMI_RTC_CACHE")
    os.environ["RSMI_RTC_CACHE"] = str(tmp_path_factory.mktemp("rtc_cache"))
    import udpspeeder_amd
    yield udpspeeder_amd
    if old is None:
        del os.environ["RSMI_RTC_CACHE"]
    else:
        os.environ["RSMI_RTC_CACHE"] = old


def test_codes_are_not_builtin():
    built = set(gen_bitslice.default_codes())
    assert not built & set(RTC_CODES)


@pytest.mark.parametrize("kn", RTC_CODES + [(20, 30), (1, 11), (100, 101)])
def test_emitters_agree(u, kn):
    assert u.bitslice_source(*kn) == gen_bitslice.emit_code(*kn)[0]


@pytest.mark.parametrize("kn", [(10, 15), (20, 30), (10, 12), (13, 23), (40, 50), (31, 36)])
def test_split_emitters_agree(u, kn):
    assert gen_bitslice.split_ok(*kn)
    assert u.bitslice_source(*kn, split=True) == gen_bitslice.emit_split(*kn)[0]


def test_split_eligibility(u):
    from udpspeeder_amd._lib import RsmiError
    for kn in [(9, 15), (10, 11), (10, 21), (20, 31)]:
        assert not gen_bitslice.split_ok(*kn)
        with pytest.raises(RsmiError):
            u.bitslice_source(*kn, split=True)


def test_row_blocks():
    assert gen_bitslice.row_blocks(10) == [(0, 10)]
    assert gen_bitslice.row_blocks(11) == [(0, 6), (6, 11)]
    assert gen_bitslice.row_blocks(30) == [(0, 10), (10, 20), (20, 30)]
    for m in range(1, 256):
        b = gen_bitslice.row_blocks(m)
        assert b[0][0] == 0 and b[-1][1] == m and all(hi - lo <= 10 for lo, hi in b)
        assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))


@pytest.fixture(scope="module")
def rtc_harness(u, tmp_path_factory):
    d = tmp_path_factory.mktemp("rtc_host")
    inc = d / "rtc_codes.inc"
    parts = [u.bitslice_source(k, n) for k, n in RTC_CODES]
    parts.append("#define BS_FOR_EACH_CODE(X) " + " ".join(f"X({k}, {n})" for k, n in RTC_CODES))
    inc.write_text("\n".join(parts) + "\n")
    exe = str(d / "bitslice_host_rtc")
    subprocess.run(["g++", "-O1", "-std=c++17", f'-DBS_HOST_INC="{inc}"', "-o", exe,
                    os.path.join(ROOT, "tests", "bitslice_host.cpp")], check=True)
    return exe


@pytest.mark.parametrize("kn", RTC_CODES)
def test_rtc_network_vs_oracle(rtc_harness, oracle, kn):
    k, n = kn
    m = n - k
    nchunks = 8
    rng = np.random.default_rng(k * 7 + n)
    data = rng.integers(0, 256, (nchunks, k, 32), dtype=np.uint8)
    data[0] = 0
    data[1] = 0xFF
    out = subprocess.run([rtc_harness], input=f"{k} {n} {nchunks}\n".encode() + data.tobytes(),
                         capture_output=True, check=True)
    par = np.frombuffer(out.stdout, np.uint8).reshape(nchunks, m, 32)
    ref = np.zeros((nchunks, n, 32), np.uint8)
    ref[:, :k] = data
    oracle.encode_batch(k, n, ref.reshape(-1), n * 32, 32, 32, nchunks)
    assert (par == ref[:, k:]).all()


def test_precompile_without_gpu(u):
    from udpspeeder_amd._lib import ENC_BITSLICE, ENC_BITSLICE_RTC
    t0 = time.time()
    u.precompile_code(10, 15)
    assert u.code_encoder(10, 15) == ENC_BITSLICE_RTC
    assert u.code_encoder(20, 30) == ENC_BITSLICE
    files = os.listdir(os.environ["RSMI_RTC_CACHE"])
    assert any(f.startswith("bs-") and f.endswith(".co") for f in files), files
    assert time.time() - t0 < 60


def test_code_object_has_no_spills(u):
    """Every kernel of the run-time code objects fits the register budget."""
    for kn in [(10, 40), (40, 60)]:
        u.precompile_code(*kn)
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not os.path.exists(readelf):
        pytest.skip("llvm-readelf absent")
    cache = os.environ["RSMI_RTC_CACHE"]
    seen = 0
    for f in os.listdir(cache):
        notes = subprocess.run([readelf, "--notes", os.path.join(cache, f)], capture_output=True,
                               text=True).stdout
        for line in notes.splitlines():
            line = line.strip()
            if line.startswith(".vgpr_spill_count:") or line.startswith(".sgpr_spill_count:"):
                assert int(line.split(":")[1]) == 0, (f, line)
                seen += 1
    assert seen >= 4


def test_precompile_rejects(u):
    from udpspeeder_amd._lib import ENC_GENERIC, ENC_NONE, RsmiError
    for kn in [(20, 30), (5, 5), (0, 3), (3, 2)]:
        with pytest.raises(RsmiError):
            u.precompile_code(*kn)
    os.environ["RSMI_RTC_MAX_COEFS"] = "8"
    try:
        with pytest.raises(RsmiError):
            u.precompile_code(9, 12)  # 27 coefficients > 8
        assert u.code_encoder(9, 12) == ENC_GENERIC
    finally:
        del os.environ["RSMI_RTC_MAX_COEFS"]
    assert u.code_encoder(5, 5) == ENC_NONE


# A process that exits while a run-time compile is inside hipRTC must exit
# cleanly and promptly: comgr/LLVM is loaded by libhiprtc on first use, so its
# static destructors are registered after (and run before) any atexit handler
# librsmi registers earlier; tearing LLVM down under a running compile crashed
# or hung the round-2 GPU test process at exit.  The library now stops
# compiles from Python's atexit and from the main thread's exit path, ahead
# of every atexit handler (bitslice_rtc.cpp shutdown_compiles).
_EXIT_PY = r"""
import os, sys, threading, time
sys.path.insert(0, {root!r})
from udpspeeder_amd._lib import lib
L = lib()
def go():
    L.rsmi_precompile_code({k}, {n})
for _ in range({threads}):
    threading.Thread(target=go, daemon=True).start()
{extra}
time.sleep({sleep})
print("main returns", flush=True)
"""

_EXIT_C = r"""
#include <pthread.h>
#include <stdio.h>
#include <unistd.h>
int rsmi_precompile_code(int k, int n);
static void *go(void *p) { (void)p; rsmi_precompile_code(40, 60); return 0; }
int main(void) {
    pthread_t t;
    pthread_create(&t, 0, go, 0);
    usleep(1500 * 1000);   /* inside hipRTC by now */
    printf("main returns\n");
    fflush(stdout);
    return 0;              /* exit() with the compile still running */
}
"""


def _run_exit(args, tmp_path, bound, expect_cached=True):
    env = dict(os.environ, RSMI_RTC_CACHE=str(tmp_path / "cold"))
    t0 = time.time()
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=bound + 60)
    dt = time.time() - t0
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "main returns" in r.stdout
    assert dt < bound, dt
    if expect_cached:
        # the compile that was inside hipRTC finished before the process went
        # away (the round-2 library exited under it: nothing cached, or SIGSEGV)
        cold = tmp_path / "cold"
        files = os.listdir(cold) if cold.exists() else []
        assert any(f.startswith("bs-") and f.endswith(".co") for f in files), files
    return dt


@pytest.mark.parametrize("case", ["one", "queue", "waiter"])
def test_exit_during_compile_python(u, tmp_path, case):
    """Interpreter exit mid-compile: a daemon thread in rsmi_precompile_code
    (40,60) (800 coefficients, ~10 s cold); 'queue' also has a 40-code -f
    table queued behind the pool; 'waiter' has six threads compiling on their
    own (caller-side compiles).  rc 0, and the exit waits for at most the
    compiles already inside hipRTC (one code each)."""
    extra = ""
    threads = 1
    if case == "queue":
        extra = ("import ctypes\n"
                 "ks = [x for x in range(11, 51)]; ns = [x + max(1, x // 2) for x in ks]\n"
                 "A = ctypes.c_int32 * len(ks)\n"
                 "assert L.rsmi_precompile_codes_async(A(*ks), A(*ns), len(ks)) >= 30\n")
    if case == "waiter":
        threads = 6
    src = _EXIT_PY.format(root=ROOT, k=40, n=60, threads=threads, extra=extra, sleep=1.5)
    _run_exit([sys.executable, "-c", src], tmp_path, bound=90)


def test_exit_during_compile_c(u, tmp_path):
    """The same from a C program linked against librsmi: main() returns while
    a pthread is inside hipRTC; the main thread's exit path waits for it."""
    c = tmp_path / "exit_mid_compile.c"
    c.write_text(_EXIT_C)
    exe = str(tmp_path / "exit_mid_compile")
    libdir = os.path.join(ROOT, "udpspeeder_amd")
    subprocess.run(["gcc", "-O1", "-o", exe, str(c), "-L" + libdir, "-lrsmi", "-lpthread",
                    "-Wl,-rpath," + libdir], check=True)
    _run_exit([exe], tmp_path, bound=90)


def test_shutdown_stops_compiles(u, tmp_path):
    """After rsmi_rtc_shutdown nothing new compiles: precompile fails and the
    code stays on the generic kernel (in a child, so this process keeps
    compiling)."""
    src = (f"import sys; sys.path.insert(0, {ROOT!r})\n"
           "from udpspeeder_amd._lib import lib, ENC_GENERIC\n"
           "L = lib(); L.rsmi_rtc_shutdown()\n"
           "assert L.rsmi_precompile_code(10, 14) != 0\n"
           "assert L.rsmi_code_encoder(10, 14) == ENC_GENERIC, L.rsmi_code_encoder(10, 14)\n"
           "print('main returns')\n")
    _run_exit([sys.executable, "-c", src], tmp_path, bound=60, expect_cached=False)


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_precompile_then_gpu_in_one_process(tmp_path):
    """rsmi_precompile_code before any GPU use, then rsmi_init, in a fresh
    process (hipRTC used to leave the shared HIP runtime without devices)."""
    env = dict(os.environ, RSMI_RTC_CACHE=str(tmp_path))
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "scripts", "precompile_then_gpu.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and "rsmi_init ok" in r.stdout, r.stdout + r.stderr


GPU_CASES = [(10, 15, 1250), (10, 15, 17), (10, 40, 1250), (5, 17, 333), (7, 9, 4000),
             (40, 60, 1280), (1, 2, 1), (2, 200, 100), (12, 20, 1250), (31, 36, 777)]


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,ln", GPU_CASES)
def test_rtc_encode_vs_oracle(gpu, oracle, u, k, n, ln):
    from udpspeeder_amd._lib import ENC_BITSLICE_RTC
    import torch
    u.wait_code(k, n)
    assert u.code_encoder(k, n) == ENC_BITSLICE_RTC
    G = 97
    S = max(16, (ln + 15) // 16 * 16) + 32
    rng = np.random.default_rng(k * 100 + n + ln)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    t = torch.from_numpy(buf).to(gpu)
    u.encode(t, k, n, ln)
    assert u.lib().rsmi_last_encoder() == ENC_BITSLICE_RTC  # the run-time kernel ran
    oracle.encode_batch(k, n, buf.reshape(-1), n * S, S, ln, G)
    out = t.cpu().numpy()
    assert (out[:, :, :ln] == buf[:, :, :ln]).all()
    pad = min(S, (ln + 127) // 128 * 128)
    assert (out[:, :, pad:] == buf[:, :, pad:]).all()


@pytest.mark.gpu
def test_rtc_ragged_plan_vs_oracle(gpu, oracle, u):
    """Build-time and run-time codes mixed in one plan: one launch for the
    build-time buckets plus one per run-time code, bit-exact."""
    import torch
    rng = np.random.default_rng(21)
    codes = [(20, 30), (3, 8), (10, 15), (5, 17), (7, 9), (1, 2)]
    G = 1500
    pick = rng.integers(0, len(codes), G)
    ks = np.array([codes[i][0] for i in pick]); ns = np.array([codes[i][1] for i in pick])
    ls = rng.integers(0, 2000, G)
    ls[:5] = [0, 1, 16, 17, 1280]
    groups, total = u.make_groups(ks, ns, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    base = torch.from_numpy(host.copy()).to(gpu)
    plan = u.rs.RaggedPlan(groups)
    assert plan.bitslice
    plan.encode(base)
    out = base.cpu().numpy()
    plan.close()
    for i in range(G):
        d = groups[i]
        seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
        oracle.encode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1)
        got = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
        assert (got[:, :d.len] == seg.reshape(d.n, d.shard_stride)[:, :d.len]).all(), i


@pytest.mark.gpu
def test_rtc_before_ready_is_generic_and_exact(gpu, oracle, u):
    """A code's first encodes run while its network compiles (generic kernel);
    the output is the same bytes before and after the switch."""
    import torch
    k, n, ln, G = 11, 19, 700, 64
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, (G, n, 704), dtype=np.uint8)
    ref = buf.copy()
    oracle.encode_batch(k, n, ref.reshape(-1), n * 704, 704, ln, G)
    t1 = torch.from_numpy(buf.copy()).to(gpu)
    u.encode(t1, k, n, ln)  # likely still compiling
    u.wait_code(k, n)
    t2 = torch.from_numpy(buf.copy()).to(gpu)
    u.encode(t2, k, n, ln)
    from udpspeeder_amd._lib import ENC_BITSLICE_RTC
    assert u.lib().rsmi_last_encoder() == ENC_BITSLICE_RTC
    for t in (t1, t2):
        assert (t.cpu().numpy()[:, :, :ln] == ref[:, :, :ln]).all()
