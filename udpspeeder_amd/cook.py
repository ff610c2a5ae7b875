"""Packet cook / de_cook on the GPU (include/rsmi_cook.h).

UDPspeeder wraps every packet it sends in ``do_cook`` (packet.cpp:303-308:
append crc32h big-endian, obscure with a random IV, XOR with the key) and
unwraps every packet it receives with ``de_cook`` (packet.cpp:310-326).  This
module exposes the batched HIP kernels of librsmi.so:

* :class:`CookContext` -- one key + flag set (the reference's ``key_string``,
  ``disable_checksum`` / ``disable_obscure`` / ``disable_xor`` globals), with
  ``cook`` / ``decook`` over torch CUDA tensors (device-resident batches, the
  production path) and ``cook_host`` / ``decook_host`` over numpy arrays.
* ``do_cook`` / ``de_cook`` -- the reference's per-packet functions with the
  reference's names, in-place semantics and return values, driven by the
  module-level globals of the same names.  They run one packet through the GPU
  (there is no CPU path).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from ._lib import (RSMI_COOK_IV_MAX, RSMI_COOK_NO_CHECKSUM, RSMI_COOK_NO_OBSCURE,
                   RSMI_COOK_NO_XOR, RsmiError, check, lib, rsmi_packet_batch)

NO_CHECKSUM, NO_OBSCURE, NO_XOR = RSMI_COOK_NO_CHECKSUM, RSMI_COOK_NO_OBSCURE, RSMI_COOK_NO_XOR
IV_MAX = RSMI_COOK_IV_MAX
TAIL_MAX = 4 + IV_MAX + 1      # bytes do_cook appends at most (crc + iv + iv_len)


def cooked_cap(length: int) -> int:
    """Bytes a packet slot needs for do_cook of `length` bytes (kernels write
    whole 16-byte pieces)."""
    return (length + TAIL_MAX + 15) // 16 * 16


def _stream_ptr(stream) -> Optional[int]:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


class CookContext:
    """A key and flag set made resident on the current device."""

    def __init__(self, key: bytes = b"", flags: int = 0):
        if isinstance(key, str):
            key = key.encode()
        if b"\0" in key:
            raise ValueError("key is a C string (key_string, misc.cpp:628): no NUL bytes")
        self.key, self.flags = bytes(key), int(flags)
        h = C.c_void_p()
        check(lib().rsmi_cook_ctx_create(self.key, self.flags, C.byref(h)), "rsmi_cook_ctx_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().rsmi_cook_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- device batches -----------------------------------------------------------
    def _batch(self, buf, lens, out_len, stride, offsets, cap, host_ok=False):
        import torch
        if not ((buf.is_cuda or (host_ok and buf.is_pinned())) and buf.dtype == torch.uint8):
            raise TypeError("buf must be a CUDA uint8 tensor")
        if lens.dtype != torch.int32 or not lens.is_cuda or not lens.is_contiguous():
            raise TypeError("lens must be a contiguous CUDA int32 tensor")
        if out_len is None:
            out_len = torch.empty_like(lens)
        n = lens.numel()
        if offsets is None and stride is None:
            stride = buf.shape[-1] if buf.dim() == 2 else None
            if stride is None:
                raise ValueError("give stride or offsets")
        if offsets is not None and (offsets.dtype != torch.int64 or not offsets.is_cuda):
            raise TypeError("offsets must be a CUDA int64 tensor")
        if offsets is None and n and (n - 1) * stride + cap > buf.numel():
            raise ValueError("batch extends past the buffer")
        b = rsmi_packet_batch(buf.data_ptr(), offsets.data_ptr() if offsets is not None else None,
                              int(stride or 0), n, int(cap), 0, lens.data_ptr(), out_len.data_ptr())
        return b, out_len

    def cook(self, buf, lens, *, cap: int, stride: Optional[int] = None, offsets=None,
             out_len=None, iv=None, iv_len=None, seed: int = 0, stream=None):
        """do_cook every packet in place; returns out_len (int32, -1 = rejected).
        iv: CUDA uint8 [count, 32] with iv_len [count], or None to draw them on
        the device from `seed`."""
        b, out_len = self._batch(buf, lens, out_len, stride, offsets, cap)
        if (iv is None) != (iv_len is None):
            raise ValueError("give both iv and iv_len or neither")
        check(lib().rsmi_cook_dev(self._h, C.byref(b), iv.data_ptr() if iv is not None else None,
                                  iv_len.data_ptr() if iv_len is not None else None,
                                  C.c_uint64(seed & (2**64 - 1)), _stream_ptr(stream)),
              "rsmi_cook_dev")
        return out_len

    def decook(self, buf, lens, *, cap: int, stride: Optional[int] = None, offsets=None,
               out_len=None, stream=None):
        """de_cook every packet in place; returns out_len (-1 where de_cook fails)."""
        b, out_len = self._batch(buf, lens, out_len, stride, offsets, cap)
        check(lib().rsmi_decook_dev(self._h, C.byref(b), _stream_ptr(stream)), "rsmi_decook_dev")
        return out_len

    @staticmethod
    def _out_ptr(out, need: int) -> int:
        import torch
        if not isinstance(out, torch.Tensor) or out.dtype != torch.uint8 or not out.is_contiguous():
            raise TypeError("out must be a contiguous uint8 tensor")
        if not out.is_cuda and not out.is_pinned():
            raise TypeError("out must be a CUDA tensor or pinned host memory")
        if out.numel() < need or out.data_ptr() % 16:
            raise ValueError(f"out must be 16-aligned with >= {need} bytes")
        return out.data_ptr()

    def _extent(self, buf, b) -> int:
        # packets sit at the same offsets in out as in buf: out spans buf
        return buf.numel()

    def cook_to(self, buf, lens, out, *, cap: int, stride: Optional[int] = None, offsets=None,
                out_len=None, iv=None, iv_len=None, seed: int = 0, stream=None):
        """do_cook every packet of buf into out at the same offset (rsmi_cook_to):
        out may be a pinned host tensor, then the cooked packets cross PCIe in
        the kernel's own stores.  Returns out_len."""
        b, out_len = self._batch(buf, lens, out_len, stride, offsets, cap)
        if (iv is None) != (iv_len is None):
            raise ValueError("give both iv and iv_len or neither")
        check(lib().rsmi_cook_to(self._h, C.byref(b), self._out_ptr(out, self._extent(buf, b)),
                                 iv.data_ptr() if iv is not None else None,
                                 iv_len.data_ptr() if iv_len is not None else None,
                                 C.c_uint64(seed & (2**64 - 1)), _stream_ptr(stream)), "rsmi_cook_to")
        return out_len

    def decook_mirror(self, buf, lens, mirror, *, cap: int, stride: Optional[int] = None, offsets=None,
                      out_len=None, stream=None):
        """de_cook every packet of buf in place and store its de-cooked bytes
        (16-byte pieces up to round_up(len, 16)) at the same offset of
        `mirror`, pinned host memory (rsmi_decook_mirror).  Returns out_len."""
        b, out_len = self._batch(buf, lens, out_len, stride, offsets, cap)
        check(lib().rsmi_decook_mirror(self._h, C.byref(b), self._out_ptr(mirror, self._extent(buf, b)),
                                       _stream_ptr(stream)), "rsmi_decook_mirror")
        return out_len

    def decook_to(self, buf, lens, out, *, cap: int, stride: Optional[int] = None, offsets=None,
                  out_len=None, stream=None):
        """de_cook every packet of buf into out at the same offset (rsmi_decook_to);
        buf may be a pinned host tensor read over PCIe in the kernel's loads."""
        import torch
        if isinstance(buf, torch.Tensor) and not buf.is_cuda:
            if not buf.is_pinned():
                raise TypeError("a host buf must be pinned")
        b, out_len = self._batch(buf, lens, out_len, stride, offsets, cap, host_ok=True)
        check(lib().rsmi_decook_to(self._h, C.byref(b), self._out_ptr(out, self._extent(buf, b)),
                                   _stream_ptr(stream)), "rsmi_decook_to")
        return out_len

    # ---- host batches -------------------------------------------------------------
    def cook_host(self, buf: np.ndarray, lens, iv=None, iv_len=None, seed: int = 0,
                  cap: Optional[int] = None) -> np.ndarray:
        """buf: [count, stride] uint8, modified in place."""
        lens = np.ascontiguousarray(lens, np.int32)
        out = np.zeros(len(lens), np.int32)
        if (iv is None) != (iv_len is None):
            raise ValueError("give both iv and iv_len or neither")
        ivp = ivlp = None
        if iv is not None:
            iv = np.ascontiguousarray(iv, np.uint8)
            iv_len = np.ascontiguousarray(iv_len, np.uint8)
            ivp, ivlp = iv.ctypes.data, iv_len.ctypes.data
        stride = buf.shape[1]
        check(lib().rsmi_cook_host(self._h, buf.ctypes.data, stride, buf.shape[0],
                                   stride if cap is None else cap, lens.ctypes.data,
                                   out.ctypes.data, ivp, ivlp, C.c_uint64(seed & (2**64 - 1))),
              "rsmi_cook_host")
        return out

    def decook_host(self, buf: np.ndarray, lens, cap: Optional[int] = None) -> np.ndarray:
        lens = np.ascontiguousarray(lens, np.int32)
        out = np.zeros(len(lens), np.int32)
        stride = buf.shape[1]
        check(lib().rsmi_decook_host(self._h, buf.ctypes.data, stride, buf.shape[0],
                                     stride if cap is None else cap, lens.ctypes.data,
                                     out.ctypes.data), "rsmi_decook_host")
        return out


# --------------------------------------------------------------------------
# The reference's per-packet interface (packet.h:42-43) and its globals
# (packet.cpp:23-28, misc.cpp:16).
key_string = b""
disable_checksum = 0
disable_obscure = 0
disable_xor = 0
_ctx_cache: dict = {}
_iv_counter = [0x5EED0F1F]


def _ctx() -> CookContext:
    flags = ((NO_CHECKSUM if disable_checksum else 0) | (NO_OBSCURE if disable_obscure else 0) |
             (NO_XOR if disable_xor else 0))
    k = (bytes(key_string), flags)
    if k not in _ctx_cache:
        _ctx_cache[k] = CookContext(*k)
    return _ctx_cache[k]


def do_cook(data: bytearray, length: int) -> int:
    """``int do_cook(char *data, int &len)``: cook data[:length] in place and
    return the new length.  `data` needs room for TAIL_MAX more bytes, as the
    reference's buf_len-sized buffers have."""
    if len(data) < length + TAIL_MAX:
        raise ValueError(f"buffer needs {length + TAIL_MAX} bytes")
    stride = cooked_cap(length)
    a = np.zeros((1, stride), np.uint8)
    a[0, :length] = np.frombuffer(bytes(data[:length]), np.uint8)
    _iv_counter[0] += 1
    out = int(_ctx().cook_host(a, [length], seed=_iv_counter[0])[0])
    if out < 0:
        raise RsmiError("do_cook rejected the packet")
    data[:out] = a[0, :out].tobytes()
    return out


def de_cook(data: bytearray, length: int):
    """``int de_cook(char *s, int &len)``: returns (ret, new_len); data is
    modified in place as the reference modifies it (also on failure)."""
    stride = (length + 15) // 16 * 16 or 16
    a = np.zeros((1, stride), np.uint8)
    a[0, :length] = np.frombuffer(bytes(data[:length]), np.uint8)
    out = int(_ctx().decook_host(a, [length])[0])
    data[:length] = a[0, :length].tobytes()
    return (0, out) if out >= 0 else (-1, length)
