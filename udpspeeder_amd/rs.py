"""Python surface of the MI355X Reed-Solomon engine.

Two layers, mirroring the reference:

* Per-group, host-buffer functions with the reference's names and semantics
  (``rs_encode2`` / ``rs_decode2`` of lib/rs.h:41,43, ``fec_new`` ... of
  lib/fec.h).  They call the reference-mangled symbols exported by
  librsmi.so (the same ones fec_manager.cpp links against), so these wrappers
  exercise exactly the drop-in C++ ABI.  A "char *data[]" is a Python list of
  writable buffers (bytearray / numpy uint8), ``None`` for a null pointer;
  ``rs_decode2`` permutes that list in place exactly as the C call permutes
  the pointer array (lib/rs.h:25-38).

* Batched, device-resident functions (``encode``, ``decode``,
  ``encode_ragged``) over torch CUDA tensors, launched on the current torch
  stream.  These are the production path: one launch covers many FEC groups.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, List, Optional, Sequence

import numpy as np

from ._lib import RSMI_OK, RsmiError, check, lib, rsmi_group


# --------------------------------------------------------------------------
# helpers
def _addr(buf) -> int:
    if isinstance(buf, np.ndarray):
        if buf.dtype != np.uint8 or not buf.flags.c_contiguous or not buf.flags.writeable:
            raise TypeError("numpy shard buffers must be writable contiguous uint8")
        return buf.ctypes.data
    if isinstance(buf, bytearray):
        return C.addressof((C.c_char * max(len(buf), 1)).from_buffer(buf)) if len(buf) else 0
    raise TypeError(f"shard buffer must be bytearray or numpy uint8, got {type(buf).__name__}")


def _ptr_array(data: Sequence) -> C.Array:
    arr = (C.c_void_p * len(data))()
    for i, b in enumerate(data):
        arr[i] = _addr(b) if b is not None else None
    return arr


def _check_sizes(data, n, size):
    if len(data) < n:
        raise ValueError(f"data has {len(data)} entries, need n={n}")
    for b in data[:n]:
        if b is not None and len(b) < size:
            raise ValueError("a shard buffer is shorter than size")


# --------------------------------------------------------------------------
# reference-interface mirror (lib/rs.h, lib/fec.h)
def rs_encode2(k: int, n: int, data: List, size: int) -> None:
    """lib/rs.h:41.  data[0..k-1] hold the data shards, data[k..n-1] are
    caller-allocated parity buffers that get overwritten."""
    _check_sizes(data, n, size)
    if any(b is None for b in data[:n]):
        raise ValueError("rs_encode2 needs all n buffers")
    lib().compat["rs_encode2"](k, n, _ptr_array(data[:n]), size)


def rs_decode2(k: int, n: int, data: List, size: int) -> int:
    """lib/rs.h:43.  data[i] is None for a missing shard.  Returns 0, -1 (fewer
    than k present) or 1; on return data[0..k-1] are the recovered data shards
    (some are former parity buffers, now overwritten), the list permuted in
    place like the C pointer array."""
    _check_sizes(data, n, size)
    arr = _ptr_array(data[:n])
    by_addr = {}
    for b in data[:n]:
        if b is not None:
            by_addr[_addr(b)] = b
    rc = lib().compat["rs_decode2"](k, n, arr, size)
    for i in range(n):
        data[i] = by_addr[arr[i]] if arr[i] else None
    return rc


def fec_new(k: int, n: int) -> Optional[int]:
    """lib/fec.h:47; returns an opaque code handle (None for invalid k/n)."""
    return lib().compat["fec_new"](k, n)


def fec_free(code: int) -> None:
    lib().compat["fec_free"](code)


def get_k(code: int) -> int:
    return lib().compat["get_k"](code)


def get_n(code: int) -> int:
    return lib().compat["get_n"](code)


def get_code(k: int, n: int) -> Optional[int]:
    return lib().compat["get_code"](k, n)


def rs_encode(code: int, data: List, size: int) -> None:
    n = get_n(code)
    _check_sizes(data, n, size)
    lib().compat["rs_encode"](code, _ptr_array(data[:n]), size)


def rs_decode(code: int, data: List, size: int) -> int:
    n = get_n(code)
    _check_sizes(data, n, size)
    arr = _ptr_array(data[:n])
    by_addr = {_addr(b): b for b in data[:n] if b is not None}
    rc = lib().compat["rs_decode"](code, arr, size)
    for i in range(n):
        data[i] = by_addr[arr[i]] if arr[i] else None
    return rc


def fec_encode(code: int, src: List, dst, index: int, sz: int) -> None:
    """lib/fec.h:50: dst = shard `index` of the code word of src[0..k-1]."""
    k = get_k(code)
    lib().compat["fec_encode"](code, _ptr_array(src[:k]), _addr(dst), index, sz)


def fec_decode(code: int, pkt: List, index: List[int], sz: int) -> int:
    """lib/fec.h:51: pkt[0..k-1] with shard indices index[0..k-1]; both lists
    are permuted in place like the C arrays."""
    k = get_k(code)
    arr = _ptr_array(pkt[:k])
    idx = (C.c_int * k)(*index[:k])
    by_addr = {_addr(b): b for b in pkt[:k] if b is not None}
    rc = lib().compat["fec_decode"](code, arr, idx, sz)
    for i in range(k):
        pkt[i] = by_addr.get(arr[i]) if arr[i] else None
        index[i] = idx[i]
    return rc


# --------------------------------------------------------------------------
# host utilities
def enc_matrix(k: int, n: int) -> np.ndarray:
    """fec_new(k,n)'s n x k systematic matrix (lib/fec.cpp:665-720)."""
    out = np.zeros((n, k), np.uint8)
    check(lib().rsmi_get_matrix(k, n, out.ctypes.data), "rsmi_get_matrix")
    return out


def decode_matrix(k: int, n: int, present: Sequence[int]):
    """(e, sel[k], miss[e], coef[e, k]) for one group; e = -1 if too few."""
    p = np.ascontiguousarray(np.asarray(present, dtype=np.uint8))
    if p.shape != (n,):
        raise ValueError("present must have n entries")
    sel = np.zeros(k, np.uint8); miss = np.zeros(k, np.uint8); coef = np.zeros(k * k, np.uint8)
    e = lib().rsmi_decode_matrix(k, n, p.ctypes.data, sel.ctypes.data, miss.ctypes.data,
                                 coef.ctypes.data)
    if e < -1:
        check(e, "rsmi_decode_matrix")
    if e < 0:
        return -1, sel, miss[:0], coef[:0].reshape(0, k)
    return e, sel, miss[:e], coef[:e * k].reshape(e, k)


def set_bitslice(enabled: bool) -> bool:
    """Use (default) or bypass the specialised bit-sliced encoders; returns
    the previous setting.  For A/B tests of the generic kernel."""
    from ._lib import RSMI_OPT_BITSLICE
    return bool(lib().rsmi_option(RSMI_OPT_BITSLICE, int(bool(enabled))))


def set_fused_decode(enabled: bool) -> bool:
    """Use (default) or bypass the fused decode kernel; returns the previous
    setting.  For A/B tests of the two-kernel (plan + apply) decode path."""
    from ._lib import RSMI_OPT_FUSED_DECODE
    return bool(lib().rsmi_option(RSMI_OPT_FUSED_DECODE, int(bool(enabled))))


def version() -> int:
    return lib().rsmi_version()


# --------------------------------------------------------------------------
# batched device API (torch CUDA tensors)
def _stream_handle(stream) -> Optional[int]:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _check_dev(t, name, dtype=None):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA tensor")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}")


def _status_out(status, G, device):
    """The caller's status tensor checked (int32, contiguous, >= G entries, on
    ``device``: the kernels write status[g] for every g < G), or a new one."""
    import torch
    if status is None:
        return torch.empty(G, dtype=torch.int32, device=device)
    _check_dev(status, "status", torch.int32)
    if status.device != device or not status.is_contiguous() or status.numel() < G:
        raise ValueError(f"status must be a contiguous int32 tensor of >= {G} entries on {device}")
    return status


def _present_bits(present_bits, G, device):
    import torch
    _check_dev(present_bits, "present_bits", torch.int32)
    if tuple(present_bits.shape) != (G, 8) or not present_bits.is_contiguous() or \
            present_bits.device != device:
        raise ValueError("present_bits must be a contiguous [G, 8] int32 tensor on the base's device")


def _shard_geometry(shards, n):
    import torch
    _check_dev(shards, "shards", torch.uint8)
    if shards.dim() != 3 or shards.shape[1] < n:
        raise ValueError("shards must be [groups, >=n, stride]")
    if shards.stride(2) != 1:
        raise ValueError("shards rows must be contiguous")
    return shards.shape[0], shards.stride(0), shards.stride(1), shards.shape[2]


def encode(shards, k: int, n: int, length: Optional[int] = None, stream=None) -> None:
    """rs_encode2 on every group of ``shards`` ([G, n, S] uint8 CUDA, S % 16 == 0):
    parity rows k..n-1 are overwritten from data rows 0..k-1."""
    G, gs, ss, S = _shard_geometry(shards, n)
    L = S if length is None else int(length)
    check(lib().rsmi_encode_dev(k, n, shards.data_ptr(), gs, ss, L, G, _stream_handle(stream)),
          "rsmi_encode_dev")


def decode(shards, present, k: int, n: int, length: Optional[int] = None, status=None,
           stream=None, placement: str = "own", slot_map=None):
    """rs_decode2 on every group: ``present`` [G, n] uint8 CUDA (nonzero =
    received).  Returns the int32 [G] status tensor (0 ok, -1 too few shards,
    1 singular).

    ``placement="own"`` (default) rebuilds each missing data row in its own
    slot.  ``placement="reference"`` writes it where fec_decode does
    (lib/fec.cpp:872-877): over the parity survivor its shuffle moves into
    data[i] (rsmi_decode_dev_ref); ``slot_map`` (uint8 [G, k] CUDA, optional)
    then receives the slot holding each data row (reference_rows reads
    through it)."""
    import torch
    G, gs, ss, S = _shard_geometry(shards, n)
    _check_dev(present, "present", torch.uint8)
    if tuple(present.shape) != (G, n) or not present.is_contiguous() or present.device != shards.device:
        raise ValueError("present must be a contiguous [G, n] uint8 tensor on the shards' device")
    status = _status_out(status, G, shards.device)
    L = S if length is None else int(length)
    if placement == "own":
        if slot_map is not None:
            raise ValueError("slot_map needs placement='reference'")
        check(lib().rsmi_decode_dev(k, n, shards.data_ptr(), gs, ss, L, G, present.data_ptr(),
                                    status.data_ptr(), _stream_handle(stream)), "rsmi_decode_dev")
    elif placement == "reference":
        mp = None
        if slot_map is not None:
            _check_dev(slot_map, "slot_map", torch.uint8)
            if tuple(slot_map.shape) != (G, k) or not slot_map.is_contiguous() or \
                    slot_map.device != shards.device:
                raise ValueError("slot_map must be a contiguous [G, k] uint8 tensor on the shards' device")
            mp = slot_map.data_ptr()
        check(lib().rsmi_decode_dev_ref(k, n, shards.data_ptr(), gs, ss, L, G, present.data_ptr(),
                                        status.data_ptr(), mp, _stream_handle(stream)),
              "rsmi_decode_dev_ref")
    else:
        raise ValueError(f"placement must be 'own' or 'reference', not {placement!r}")
    return status


def reference_rows(shards, slot_map):
    """The k data rows of every group after a reference-placement decode, in
    data[] order: shards[g, slot_map[g, i]] (a [G, k, S] gather, on the
    device)."""
    import torch
    G = shards.shape[0]
    gi = torch.arange(G, device=shards.device).unsqueeze(1)
    return shards[gi, slot_map.long()]


def ref_slot_map(k: int, n: int, present) -> np.ndarray:
    """Host slot map of one group (rsmi_ref_slot_map): the slot holding data
    row i after rs_decode2, the permutation fec_decode's shuffle leaves in
    data[0..k-1] (0xFF: erased row of a group with too few shards)."""
    pres = np.ascontiguousarray(np.asarray(present, np.uint8).reshape(-1)[:n])
    out = np.zeros(k, np.uint8)
    rc = lib().rsmi_ref_slot_map(k, n, pres.ctypes.data, out.ctypes.data)
    if rc < -1:
        raise RsmiError(f"rsmi_ref_slot_map failed ({rc})")
    return out


def make_groups(ks: Iterable[int], ns: Iterable[int], lens: Iterable[int],
                align: int = 16):
    """Pack a ragged batch: returns (descriptor array, total bytes).  Each
    group's shards are contiguous with stride round_up(len, align)."""
    ks = np.asarray(list(ks), np.int64); ns = np.asarray(list(ns), np.int64)
    ls = np.asarray(list(lens), np.int64)
    ss = np.maximum((ls + align - 1) // align * align, align)
    sizes = ss * ns
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]) if len(sizes) else np.zeros(0, np.int64)
    arr = (rsmi_group * len(ks))()
    for i in range(len(ks)):
        arr[i] = rsmi_group(int(offs[i]), int(ss[i]), int(ls[i]), int(ks[i]), int(ns[i]), 0)
    return arr, int(sizes.sum()) if len(sizes) else 0


_GROUP_DT = np.dtype([("offset", "<u8"), ("shard_stride", "<u4"), ("len", "<u4"),
                      ("k", "<u2"), ("n", "<u2"), ("reserved", "<u4")])  # rsmi_group, 24 B


def encode_ragged(base, groups, stream=None) -> None:
    """Encode a ragged batch in one launch.  ``base`` is a 1-D uint8 CUDA tensor,
    ``groups`` a ctypes rsmi_group array from make_groups (host)."""
    import torch
    _check_dev(base, "base", torch.uint8)
    check(lib().rsmi_encode_ragged(C.cast(groups, C.c_void_p), len(groups), base.data_ptr(),
                                   _stream_handle(stream)), "rsmi_encode_ragged")


class RaggedPlan:
    """A device-resident plan for one ragged batch layout (rsmi_ragged_plan)."""

    def __init__(self, groups, wait_codes: bool = True):
        """``wait_codes``: first wait for the run-time bit-sliced networks of
        the batch's codes (rsmi_wait_code), so the plan takes the bit-sliced
        path; False makes the plan at once (generic kernel for a batch with a
        code still compiling)."""
        self._h = C.c_void_p()
        self.ngroups = len(groups)
        if wait_codes and self.ngroups:
            arr = np.frombuffer(bytes(groups), dtype=_GROUP_DT)
            for k, n in sorted(set(zip(arr["k"].tolist(), arr["n"].tolist()))):
                check(lib().rsmi_wait_code(k, n), "rsmi_wait_code")
        check(lib().rsmi_ragged_plan_create(C.cast(groups, C.c_void_p), len(groups),
                                            C.byref(self._h)), "rsmi_ragged_plan_create")

    @property
    def bitslice(self) -> bool:
        return bool(lib().rsmi_ragged_plan_uses_bitslice(self._h))

    def encode(self, base, stream=None) -> None:
        _check_dev(base, "base")
        check(lib().rsmi_encode_ragged_plan(self._h, base.data_ptr(), _stream_handle(stream)),
              "rsmi_encode_ragged_plan")

    def decode(self, base, present_bits, status=None, stream=None, placement: str = "own",
               slot_map=None):
        """rs_decode2 on every group of the plan's layout; ``present_bits`` an
        int32 [G, 8] CUDA tensor of 256-bit masks (synth.present_bits).
        ``placement="reference"`` writes rebuilt rows where fec_decode does
        (rsmi_decode_ragged_plan_ref); ``slot_map`` (uint8 [G, S] CUDA,
        optional) then receives each group's first min(k, S) slot-map entries.
        Returns the int32 [G] status tensor."""
        import torch
        _check_dev(base, "base")
        _present_bits(present_bits, self.ngroups, base.device)
        status = _status_out(status, self.ngroups, base.device)
        if placement == "own":
            if slot_map is not None:
                raise ValueError("slot_map needs placement='reference'")
            check(lib().rsmi_decode_ragged_plan(self._h, base.data_ptr(), present_bits.data_ptr(),
                                                status.data_ptr(), _stream_handle(stream)),
                  "rsmi_decode_ragged_plan")
        elif placement == "reference":
            mp, ms = None, 0
            if slot_map is not None:
                _check_dev(slot_map, "slot_map", torch.uint8)
                if slot_map.dim() != 2 or slot_map.shape[0] != self.ngroups or \
                        not slot_map.is_contiguous() or slot_map.device != base.device:
                    raise ValueError("slot_map must be a contiguous [G, S] uint8 tensor on the base's device")
                mp, ms = slot_map.data_ptr(), slot_map.shape[1]
            check(lib().rsmi_decode_ragged_plan_ref(self._h, base.data_ptr(), present_bits.data_ptr(),
                                                    status.data_ptr(), mp, ms, _stream_handle(stream)),
                  "rsmi_decode_ragged_plan_ref")
        else:
            raise ValueError(f"placement must be 'own' or 'reference', not {placement!r}")
        return status

    def close(self) -> None:
        if self._h:
            import torch
            torch.cuda.synchronize()
            lib().rsmi_ragged_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            if self._h:
                lib().rsmi_ragged_plan_destroy(self._h)
        except Exception:
            pass


def encode_ragged_dev(base, dev_groups, ngroups: int, stream=None) -> None:
    """Graph-capturable ragged encode with a device descriptor tensor (uint8,
    24 bytes per group); codes must be resident (prepare_code)."""
    check(lib().rsmi_encode_ragged_dev(dev_groups.data_ptr(), ngroups, base.data_ptr(),
                                       _stream_handle(stream)), "rsmi_encode_ragged_dev")


def decode_ragged_dev(base, dev_groups, ngroups: int, present_bits, status=None, kmax: int = 64,
                      stream=None):
    """Graph-capturable ragged decode with a device descriptor tensor (24
    bytes per group); codes must be resident (prepare_code).  Returns status."""
    import torch
    _check_dev(base, "base", torch.uint8)
    _check_dev(dev_groups, "dev_groups", torch.uint8)
    if dev_groups.device != base.device or not dev_groups.is_contiguous() or \
            dev_groups.numel() < 24 * ngroups:
        raise ValueError(f"dev_groups must be a contiguous uint8 tensor of >= {24 * ngroups} bytes")
    _present_bits(present_bits, ngroups, base.device)
    status = _status_out(status, ngroups, base.device)
    check(lib().rsmi_decode_ragged_dev(dev_groups.data_ptr(), ngroups, base.data_ptr(),
                                       present_bits.data_ptr(), status.data_ptr(), kmax,
                                       _stream_handle(stream)), "rsmi_decode_ragged_dev")
    return status


def decode_ragged(base, groups, present_bits, status=None, stream=None):
    """rs_decode2 on every group of a ragged batch described by a host ctypes
    rsmi_group array (make_groups); synchronous.  Returns status."""
    import torch
    _check_dev(base, "base", torch.uint8)
    _present_bits(present_bits, len(groups), base.device)
    status = _status_out(status, len(groups), base.device)
    check(lib().rsmi_decode_ragged(C.cast(groups, C.c_void_p), len(groups), base.data_ptr(),
                                   present_bits.data_ptr(), status.data_ptr(),
                                   _stream_handle(stream)), "rsmi_decode_ragged")
    return status


def prepare_code(k: int, n: int) -> None:
    check(lib().rsmi_prepare_code(k, n), "rsmi_prepare_code")


def wait_code(k: int, n: int) -> None:
    """prepare_code, then wait for the (k,n) run-time bit-sliced network (if
    the code gets one) and load it on the current device."""
    check(lib().rsmi_wait_code(k, n), "rsmi_wait_code")


def precompile_code(k: int, n: int) -> None:
    """Compile the run-time network of (k,n) now (no GPU needed); raises
    RsmiError for codes that get none (built-in, n == k, too large)."""
    check(lib().rsmi_precompile_code(k, n), "rsmi_precompile_code")


def code_encoder(k: int, n: int) -> int:
    """Which encoder (k,n) runs now: _lib.ENC_* (generic, build-time bit-sliced,
    run-time bit-sliced, still compiling)."""
    r = lib().rsmi_code_encoder(k, n)
    if r < 0:
        check(r, "rsmi_code_encoder")
    return r


def bitslice_source(k: int, n: int, split: bool = False) -> str:
    """The XOR-network source of (k,n) as emitted for hipRTC (split=True: the
    two-wave split-k form)."""
    L = lib()
    fn = L.rsmi_bitslice_split_source if split else L.rsmi_bitslice_source
    size = fn(k, n, None, 0)
    if size < 0:
        check(int(size), fn.__name__)
    buf = C.create_string_buffer(size + 1)
    fn(k, n, buf, size + 1)
    return buf.value.decode()


def reserve(k: int, n: int, ngroups: int, stream=None) -> None:
    check(lib().rsmi_reserve(k, n, ngroups, _stream_handle(stream)), "rsmi_reserve")


def fill_data(shards, k: int, length: int, seed: int, g0: int = 0, stream=None) -> None:
    """Synthetic SplitMix64 data into rows 0..k-1 of [G, n, S] ``shards``."""
    G, gs, ss, S = _shard_geometry(shards, k)
    check(lib().rsmi_fill_data(k, length, shards.data_ptr(), gs, ss, g0, G,
                               C.c_uint64(seed & (2**64 - 1)), _stream_handle(stream)),
          "rsmi_fill_data")


def fill_data_flat(base, k: int, length: int, offset: int, group_stride: int, shard_stride: int,
                   g0: int, ngroups: int, seed: int, stream=None) -> None:
    check(lib().rsmi_fill_data(k, length, base.data_ptr() + offset, group_stride, shard_stride,
                               g0, ngroups, C.c_uint64(seed & (2**64 - 1)),
                               _stream_handle(stream)), "rsmi_fill_data")


def encode_pinned(data, parity, k: int, n: int, length: int, chunk_groups: int = 4096) -> None:
    """End-to-end encode from host memory: ``data`` [G, k, S] and ``parity``
    [G, n-k, S] uint8 CPU tensors/arrays (pin them for overlap); chunks are
    pipelined H2D -> encode -> D2H inside the library."""
    def geo(x):
        if hasattr(x, "data_ptr"):
            return x.data_ptr(), x.stride(0), x.stride(1), x.shape
        return x.ctypes.data, x.strides[0], x.strides[1], x.shape
    dp, dgs, dss, dsh = geo(data)
    pp, pgs, pss, psh = geo(parity)
    if dss != pss or dsh[0] != psh[0] or dsh[1] != k or psh[1] != n - k:
        raise ValueError("data [G,k,S] and parity [G,n-k,S] must share G and S")
    check(lib().rsmi_encode_pinned(k, n, dp, dgs, pp, pgs, dss, length, dsh[0], chunk_groups),
          "rsmi_encode_pinned")


def decode_pinned(shards, present, k: int, n: int, length: int, chunk_groups: int = 4096):
    """End-to-end decode from host memory: ``shards`` [G, n, S] uint8 CPU
    tensor/array (pin it for overlap), ``present`` [G, n]; missing data rows
    are rebuilt in place.  Returns the int32 [G] status array."""
    if hasattr(shards, "data_ptr"):
        sp, gs, ss, sh = shards.data_ptr(), shards.stride(0), shards.stride(1), shards.shape
    else:
        sp, gs, ss, sh = shards.ctypes.data, shards.strides[0], shards.strides[1], shards.shape
    pres = np.ascontiguousarray(np.asarray(present), dtype=np.uint8)
    if pres.shape != (sh[0], n):
        raise ValueError("present must be [G, n]")
    st = np.zeros(sh[0], np.int32)
    check(lib().rsmi_decode_pinned(k, n, sp, gs, ss, length, sh[0], pres.ctypes.data,
                                   st.ctypes.data, chunk_groups), "rsmi_decode_pinned")
    return st


def _host_ptr(x):
    return x.data_ptr() if hasattr(x, "data_ptr") else x.ctypes.data


def encode_ragged_pinned(host_base, groups, chunk_groups: int = 8192) -> None:
    """rsmi_encode_ragged_pinned: a ragged batch (``groups`` from make_groups,
    ascending offsets) in host memory ``host_base`` (uint8 CPU tensor/array;
    pin it for overlap): parity rows written in place, chunks pipelined
    H2D -> encode -> D2H (split by n*len over the device list, if one is set)."""
    check(lib().rsmi_encode_ragged_pinned(groups, len(groups), _host_ptr(host_base), chunk_groups),
          "rsmi_encode_ragged_pinned")


def decode_ragged_pinned(host_base, groups, present_bits, chunk_groups: int = 8192):
    """rsmi_decode_ragged_pinned: missing data rows of every group rebuilt in
    place in host memory; ``present_bits`` uint32/int32 [G, 8] host array
    (synth.present_bits).  Returns the int32 [G] status array."""
    bits = np.ascontiguousarray(np.asarray(present_bits).view(np.uint32))
    if bits.shape != (len(groups), 8):
        raise ValueError("present_bits must be [G, 8]")
    st = np.zeros(len(groups), np.int32)
    check(lib().rsmi_decode_ragged_pinned(groups, len(groups), _host_ptr(host_base), bits.ctypes.data,
                                          st.ctypes.data, chunk_groups), "rsmi_decode_ragged_pinned")
    return st


def set_devices(devices) -> None:
    """rsmi_use_devices: split the host-memory batch entry points
    (encode_pinned / decode_pinned) over these devices, one contiguous group
    range each (a device may repeat); [] restores the current device."""
    d = np.ascontiguousarray(np.asarray(list(devices), np.int32))
    check(lib().rsmi_use_devices(d.ctypes.data if d.size else None, int(d.size)), "rsmi_use_devices")


def get_devices():
    n = lib().rsmi_get_devices(None, 0)
    out = np.zeros(max(n, 1), np.int32)
    lib().rsmi_get_devices(out.ctypes.data, n)
    return [int(x) for x in out[:n]]


def split_ranges(n: int, parts: int, cost=None):
    """rsmi_split_ranges: [(start, end)] of `parts` contiguous ranges over n
    items -- near-equal counts, or near-equal summed cost."""
    b = np.zeros(parts + 1, np.int64)
    c = None if cost is None else np.ascontiguousarray(np.asarray(cost, np.int64))
    if c is not None and c.size != n:
        raise ValueError("cost must have n entries")
    check(lib().rsmi_split_ranges(int(n), c.ctypes.data if c is not None and c.size else None, int(parts),
                                  b.ctypes.data), "rsmi_split_ranges")
    return [(int(b[i]), int(b[i + 1])) for i in range(parts)]


def groups_to_device(groups, device="cuda"):
    """Copy a ctypes rsmi_group array to a device uint8 tensor (24 B/group)."""
    import torch
    raw = np.frombuffer(bytes(groups), np.uint8).copy()
    return torch.from_numpy(raw).to(device)


def fill_ragged(base, dev_groups, ngroups: int, seed: int, g0: int = 0, stream=None) -> None:
    check(lib().rsmi_fill_ragged(dev_groups.data_ptr(), ngroups, base.data_ptr(), g0,
                                 C.c_uint64(seed & (2**64 - 1)), _stream_handle(stream)),
          "rsmi_fill_ragged")


# host-memory batched helpers (pinned staging inside the library)
def encode_host(buf: np.ndarray, k: int, n: int, length: int, group_stride: int,
                shard_stride: int, ngroups: int) -> None:
    check(lib().rsmi_encode_host(k, n, buf.ctypes.data, group_stride, shard_stride, length,
                                 ngroups), "rsmi_encode_host")


def decode_host(buf: np.ndarray, present: np.ndarray, k: int, n: int, length: int,
                group_stride: int, shard_stride: int, ngroups: int) -> np.ndarray:
    pres = np.ascontiguousarray(present, dtype=np.uint8)
    st = np.zeros(ngroups, np.int32)
    check(lib().rsmi_decode_host(k, n, buf.ctypes.data, group_stride, shard_stride, length,
                                 ngroups, pres.ctypes.data, st.ctypes.data), "rsmi_decode_host")
    return st
