"""Locate and bind librsmi.so (built in-tree by ``make -C udpspeeder_amd/csrc``).

The product path has no fallback: if the shared library is missing this
module raises at import of any compute entry point, and every GPU entry point
reports HIP errors (no device, launch failure) as exceptions.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RSMI_LIB", os.path.join(_HERE, "librsmi.so"))

RSMI_OK = 0
RSMI_ERR_INVALID = -2
RSMI_ERR_HIP = -3
RSMI_ERR_NOMEM = -4
RSMI_OPT_BITSLICE = 1
RSMI_OPT_FUSED_DECODE = 2
RSMI_OPT_ONE_GROUP = 3
RSMI_OPT_CLS_REC_CAP = 4
RSMI_OPT_ONE_SERVER = 5
RSMI_OPT_ONE_SERVER_LIFE = 6
RSMI_OPT_PARITY_COOK = 7
RSMI_DEC_OK = 0
RSMI_DEC_TOO_FEW = -1
RSMI_DEC_SINGULAR = 1
RSMI_DEC_UNSUPPORTED = 2

# Mangled C++ names of the drop-in surface (include/rs_compat.h); these are the
# exact symbols the reference's objects link against (lib/rs.h, lib/fec.h).
MANGLED = {
    "rs_encode2": "_Z10rs_encode2iiPPci",
    "rs_decode2": "_Z10rs_decode2iiPPci",
    "rs_encode": "_Z9rs_encodePvPPci",
    "rs_decode": "_Z9rs_decodePvPPci",
    "get_code": "_Z8get_codeii",
    "fec_new": "_Z7fec_newii",
    "fec_free": "_Z8fec_freePv",
    "fec_encode": "_Z10fec_encodePvPS_S_ii",
    "fec_decode": "_Z10fec_decodePvPS_Pii",
    "get_k": "_Z5get_kPv",
    "get_n": "_Z5get_nPv",
}


class RsmiError(RuntimeError):
    pass


class rsmi_group(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("shard_stride", C.c_uint32), ("len", C.c_uint32),
                ("k", C.c_uint16), ("n", C.c_uint16), ("reserved", C.c_uint32)]


class rsmi_packet_batch(C.Structure):  # include/rsmi_cook.h
    _fields_ = [("base", C.c_void_p), ("offset", C.c_void_p), ("stride", C.c_int64),
                ("count", C.c_int64), ("cap", C.c_int32), ("reserved", C.c_int32),
                ("len", C.c_void_p), ("out_len", C.c_void_p)]


class rsmi_fec_config(C.Structure):  # include/rsmi_fec.h
    _fields_ = [("mode", C.c_int32), ("mtu", C.c_int32), ("queue_len", C.c_int32),
                ("short_packet_optimize", C.c_int32), ("header_overhead", C.c_int32),
                ("rs_cnt", C.c_int32), ("rs_y", C.c_uint8 * 256)]


class rsmi_fenc_packet(C.Structure):
    _fields_ = [("slot", C.c_int64), ("len", C.c_int32), ("event", C.c_int32)]


# encoder kinds (rsmi_code_encoder)
ENC_NONE, ENC_GENERIC, ENC_BITSLICE, ENC_BITSLICE_RTC, ENC_COMPILING = 0, 1, 2, 3, 4

RSMI_COOK_NO_CHECKSUM, RSMI_COOK_NO_OBSCURE, RSMI_COOK_NO_XOR = 1, 2, 4
RSMI_COOK_IV_MAX = 32
RSMI_COOK_MAX_LEN = 65535


_lock = threading.Lock()
_lib = None


def _bind(lib: C.CDLL) -> C.CDLL:
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int
    sig = {
        "rsmi_version": ([], i32),
        "rsmi_option": ([i32, i32], i32),
        "rsmi_dropin_latency": ([i32, i32, i32, i32, vp, i32, vp], i32),
        "rsmi_init": ([], i32),
        "rsmi_quiesce": ([], i32),
        "rsmi_last_error": ([], C.c_char_p),
        "rsmi_get_matrix": ([i32, i32, vp], i32),
        "rsmi_decode_matrix": ([i32, i32, vp, vp, vp, vp], i32),
        "rsmi_prepare_code": ([i32, i32], i32),
        "rsmi_reserve": ([i32, i32, i64, vp], i32),
        "rsmi_code_encoder": ([i32, i32], i32),
        "rsmi_last_encoder": ([], i32),
        "rsmi_wait_code": ([i32, i32], i32),
        "rsmi_precompile_code": ([i32, i32], i32),
        "rsmi_rtc_shutdown": ([], None),
        "rsmi_precompile_codes_async": ([vp, vp, i32], i32),
        "rsmi_bitslice_source": ([i32, i32, C.c_char_p, i64], i64),
        "rsmi_bitslice_split_source": ([i32, i32, C.c_char_p, i64], i64),
        "rsmi_encode_dev": ([i32, i32, vp, i64, i64, i32, i64, vp], i32),
        "rsmi_decode_dev": ([i32, i32, vp, i64, i64, i32, i64, vp, vp, vp], i32),
        "rsmi_decode_dev_ref": ([i32, i32, vp, i64, i64, i32, i64, vp, vp, vp, vp], i32),
        "rsmi_ref_slot_map": ([i32, i32, vp, vp], i32),
        "rsmi_encode_ragged": ([vp, i64, vp, vp], i32),
        "rsmi_encode_ragged_dev": ([vp, i64, vp, vp], i32),
        "rsmi_encode_host": ([i32, i32, vp, i64, i64, i32, i64], i32),
        "rsmi_decode_host": ([i32, i32, vp, i64, i64, i32, i64, vp, vp], i32),
        "rsmi_fill_data": ([i32, i32, vp, i64, i64, i64, i64, C.c_uint64, vp], i32),
        "rsmi_copy_peak": ([vp, vp, i64, i32, vp], i32),
        "rsmi_fill_ragged": ([vp, i64, vp, i64, C.c_uint64, vp], i32),
        "rsmi_ragged_plan_create": ([vp, i64, vp], i32),
        "rsmi_encode_ragged_plan": ([vp, vp, vp], i32),
        "rsmi_ragged_plan_uses_bitslice": ([vp], i32),
        "rsmi_ragged_plan_destroy": ([vp], None),
        "rsmi_decode_ragged_plan": ([vp, vp, vp, vp, vp], i32),
        "rsmi_decode_ragged_plan_ref": ([vp, vp, vp, vp, vp, i32, vp], i32),
        "rsmi_decode_ragged_dev_ref": ([vp, i64, vp, vp, vp, i32, vp, i32, vp], i32),
        "rsmi_decode_ragged_dev": ([vp, i64, vp, vp, vp, i32, vp], i32),
        "rsmi_decode_ragged": ([vp, i64, vp, vp, vp, vp], i32),
        "rsmi_encode_pinned": ([i32, i32, vp, i64, vp, i64, i64, i32, i64, i64], i32),
        "rsmi_decode_pinned": ([i32, i32, vp, i64, i64, i32, i64, vp, vp, i64], i32),
        "rsmi_last_decode_pinned_path": ([], i32),
        "rsmi_encode_ragged_pinned": ([vp, i64, vp, i64], i32),
        "rsmi_decode_ragged_pinned": ([vp, i64, vp, vp, vp, i64], i32),
        "rsmi_use_devices": ([vp, i32], i32),
        "rsmi_get_devices": ([vp, i32], i32),
        "rsmi_split_ranges": ([i64, vp, i32, vp], i32),
        "rsmi_cook_ctx_create": ([C.c_char_p, i32, vp], i32),
        "rsmi_cook_ctx_destroy": ([vp], None),
        "rsmi_cook_dev": ([vp, vp, vp, vp, C.c_uint64, vp], i32),
        "rsmi_decook_dev": ([vp, vp, vp], i32),
        "rsmi_cook_to": ([vp, vp, vp, vp, vp, C.c_uint64, vp], i32),
        "rsmi_decook_to": ([vp, vp, vp, vp], i32),
        "rsmi_decook_mirror": ([vp, vp, vp, vp], i32),
        "rsmi_cook_host": ([vp, vp, i64, i64, C.c_int32, vp, vp, vp, vp, C.c_uint64], i32),
        "rsmi_decook_host": ([vp, vp, i64, i64, C.c_int32, vp, vp], i32),
        "rsmi_fec_config_init": ([vp, C.c_char_p, i32, i32, i32], i32),
        "rsmi_fenc_create": ([vp, C.c_uint32, vp], i32),
        "rsmi_fenc_next_config": ([vp, vp], i32),
        "rsmi_fenc_destroy": ([vp], None),
        "rsmi_fenc_plan": ([vp, i64, vp, vp, vp, vp, vp, vp, vp], i32),
        "rsmi_fenc_packets": ([vp, vp], i32),
        "rsmi_fenc_groups": ([vp, vp, vp, vp, vp, vp, vp], i32),
        "rsmi_fenc_packet_runs": ([vp, vp, vp], i32),
        "rsmi_fenc_run_dev": ([vp, vp, i64, vp], i32),
        "rsmi_fenc_run_cooked_dev": ([vp, vp, i64, vp, C.c_uint64, vp, vp, vp], i32),
        "rsmi_fenc_run_cooked_packed_dev": ([vp, vp, i64, vp, C.c_uint64, vp, i64, vp, vp], i32),
        "rsmi_fenc_last_parity_cooked": ([vp], i64),
        "rsmi_fcol_create": ([vp], i32),
        "rsmi_fcol_destroy": ([vp], None),
        "rsmi_debug_fcol_fail": ([i32], i32),
        "rsmi_fenc_run_many": ([vp, vp, C.c_int32, vp, i64, vp, C.c_uint64, vp, vp, vp], i32),
        "rsmi_fenc_plan_many": ([vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32], i32),
        "rsmi_fdec_plan_many": ([vp, i32, vp, vp, vp, vp, vp, i64, vp, vp, i32], i32),
        "rsmi_fdcol_create": ([vp], i32),
        "rsmi_fdcol_destroy": ([vp], None),
        "rsmi_fdec_run_many": ([vp, vp, C.c_int32, vp], i32),
        "rsmi_fdec_create": ([C.c_int32, vp], i32),
        "rsmi_fdec_destroy": ([vp], None),
        "rsmi_fdec_plan": ([vp, i64, vp, vp, vp, vp, i64, vp, vp], i32),
        "rsmi_fdec_run_dev": ([vp, vp], i32),
        "rsmi_fdec_outputs": ([vp, vp], i32),
        "rsmi_fdec_output_list": ([vp, vp, vp, vp], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    m = {k: getattr(lib, v) for k, v in MANGLED.items()}
    m["rs_encode2"].argtypes = [i32, i32, vp, i32]; m["rs_encode2"].restype = None
    m["rs_decode2"].argtypes = [i32, i32, vp, i32]; m["rs_decode2"].restype = i32
    m["rs_encode"].argtypes = [vp, vp, i32]; m["rs_encode"].restype = None
    m["rs_decode"].argtypes = [vp, vp, i32]; m["rs_decode"].restype = i32
    m["get_code"].argtypes = [i32, i32]; m["get_code"].restype = vp
    m["fec_new"].argtypes = [i32, i32]; m["fec_new"].restype = vp
    m["fec_free"].argtypes = [vp]; m["fec_free"].restype = None
    m["fec_encode"].argtypes = [vp, vp, vp, i32, i32]; m["fec_encode"].restype = None
    m["fec_decode"].argtypes = [vp, vp, vp, i32]; m["fec_decode"].restype = i32
    m["get_k"].argtypes = [vp]; m["get_k"].restype = i32
    m["get_n"].argtypes = [vp]; m["get_n"].restype = i32
    lib.compat = m
    return lib


def lib() -> C.CDLL:
    """The loaded librsmi.so (raises RsmiError if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RsmiError(
                    f"{LIB_PATH} not found: build it with `make -C udpspeeder_amd/csrc` "
                    "(or __graft_entry__.build()); there is no CPU fallback")
            _share_torch_hip_runtime()
            _lib = _bind(C.CDLL(LIB_PATH))
            # run-time compiles still inside hipRTC finish before the
            # interpreter (and then comgr/LLVM) tears down (bitslice_rtc.cpp)
            atexit.register(_lib.rsmi_rtc_shutdown)
        return _lib


def _share_torch_hip_runtime() -> None:
    """Load torch's HIP runtime before librsmi, so the process has ONE.

    librsmi.so needs libamdhip64.so.7; torch's ROCm libraries need the
    unversioned libamdhip64.so from torch/lib.  Loaded first, librsmi pulls in
    /opt/rocm's runtime and torch later maps its own copy: two HIP runtimes
    (two ROCr instances) in one process, and only the one that initialises
    first sees the GPU -- rsmi_init then fails with "no ROCm-capable device"
    behind a working torch, or torch.cuda.is_available() turns False
    (scripts/rt_order_probe.py on the GPU box).  With torch imported first,
    librsmi's libamdhip64.so.7 resolves to torch's already-loaded runtime
    (same SONAME).  Without torch installed there is only one runtime anyway.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def check(rc: int, what: str) -> None:
    if rc != RSMI_OK:
        msg = lib().rsmi_last_error().decode(errors="replace")
        raise RsmiError(f"{what} failed ({rc}): {msg}")
