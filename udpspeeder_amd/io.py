"""Batched UDP socket I/O into slot slabs (include/rsmi_io.h).

UDPspeeder reads and writes one datagram per system call (recvfrom / recv in
tunnel_client.cpp:47,119, sendto / send in my_send, packet.cpp:149-231).  These
move a batch per call (recvmmsg / sendmmsg) between a socket and a slab of
fixed-size slots in pinned host memory, the layout the FEC managers and cook
kernels use, so each batch crosses PCIe in one copy.
"""
import ctypes as C
import socket
import struct

import numpy as np

from ._lib import check, lib


class rsmi_udp_addr(C.Structure):
    _fields_ = [("storage", C.c_uint8 * 128), ("len", C.c_uint32), ("reserved", C.c_uint32)]


def _bind(L):
    if getattr(L, "_io_bound", False):
        return L
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    L.rsmi_host_alloc.argtypes = [i64, C.POINTER(vp)]
    L.rsmi_host_alloc.restype = C.c_int
    L.rsmi_host_free.argtypes = [vp]
    L.rsmi_host_free.restype = None
    L.rsmi_udp_recv_batch.argtypes = [C.c_int, vp, i64, i64, i32, i32, i32, vp, vp]
    L.rsmi_udp_recv_batch.restype = C.c_int
    L.rsmi_udp_send_batch.argtypes = [C.c_int, vp, i64, i64, vp, vp, i32, vp]
    L.rsmi_udp_send_batch.restype = C.c_int
    L.rsmi_udp_send_ptrs.argtypes = [C.c_int, vp, vp, i32, vp]
    L.rsmi_udp_send_ptrs.restype = C.c_int
    L._io_bound = True
    return L


def addr_of(host: str, port: int) -> rsmi_udp_addr:
    """An IPv4 sockaddr_in for (host, port)."""
    a = rsmi_udp_addr()
    raw = struct.pack("=H", socket.AF_INET) + struct.pack("!H", port) + socket.inet_aton(host) + bytes(8)
    C.memmove(a.storage, raw, len(raw))
    a.len = len(raw)
    return a


def addr_to_tuple(a: rsmi_udp_addr):
    raw = bytes(a.storage[:a.len])
    fam = struct.unpack("=H", raw[:2])[0]
    if fam != socket.AF_INET:
        return None
    return socket.inet_ntoa(raw[4:8]), struct.unpack("!H", raw[2:4])[0]


class Slab:
    """`nslots` slots of `slot_stride` bytes in pinned host memory (a numpy view)."""

    def __init__(self, nslots: int, slot_stride: int):
        L = _bind(lib())
        self.nslots, self.stride = nslots, slot_stride
        p = C.c_void_p()
        check(L.rsmi_host_alloc(nslots * slot_stride, C.byref(p)), "rsmi_host_alloc")
        self._p = p
        self.buf = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (nslots * slot_stride,))

    @property
    def ptr(self) -> int:
        return self._p.value

    def slot(self, i: int, off: int = 0, n: int = None) -> np.ndarray:
        a = i * self.stride + off
        return self.buf[a:a + (self.stride - off if n is None else n)]

    def close(self):
        if getattr(self, "_p", None) and self._p.value:
            lib().rsmi_host_free(self._p)
            self._p = None
            self.buf = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def recv_batch(sock, slab: Slab, slot_off: int, max_len: int, max_pkts: int, timeout_ms: int = -1,
               with_addr: bool = False):
    """Datagrams from `sock` into slots 0.. of `slab`; returns lens (int32, -1 =
    longer than max_len, dropped as the reference drops it) [and senders]."""
    L = _bind(lib())
    lens = np.zeros(max(1, max_pkts), np.int32)
    addrs = (rsmi_udp_addr * max(1, max_pkts))() if with_addr else None
    n = L.rsmi_udp_recv_batch(sock.fileno(), slab.ptr, slab.stride, slot_off, max_len, max_pkts,
                              timeout_ms, lens.ctypes.data, C.cast(addrs, C.c_void_p) if addrs else None)
    check(min(n, 0), "rsmi_udp_recv_batch")
    if with_addr:
        return lens[:n], [addrs[i] for i in range(n)]
    return lens[:n]


def send_batch(sock, slab: Slab, slot_off: int, lens, slots=None, to: rsmi_udp_addr = None) -> int:
    """Send datagram i (lens[i] bytes at slot slots[i], or slot i) to `to` (or
    the connected peer); lens < 0 are skipped.  Returns the number sent."""
    L = _bind(lib())
    lens = np.ascontiguousarray(lens, np.int32)
    sl = None if slots is None else np.ascontiguousarray(slots, np.int64)
    n = L.rsmi_udp_send_batch(sock.fileno(), slab.ptr, slab.stride, slot_off,
                              sl.ctypes.data if sl is not None else None, lens.ctypes.data,
                              len(lens), C.byref(to) if to is not None else None)
    check(min(n, 0), "rsmi_udp_send_batch")
    return n


def send_ptrs(sock, ptrs, lens, to: rsmi_udp_addr = None) -> int:
    """Send datagram i = lens[i] bytes at host address ptrs[i] (e.g. the FEC
    decoder's outputs_raw()); lens < 0 are skipped.  Returns the number sent."""
    L = _bind(lib())
    p = np.ascontiguousarray(ptrs, np.uint64)
    lens = np.ascontiguousarray(lens, np.int32)
    n = L.rsmi_udp_send_ptrs(sock.fileno(), p.ctypes.data, lens.ctypes.data, len(lens),
                             C.byref(to) if to is not None else None)
    check(min(n, 0), "rsmi_udp_send_ptrs")
    return n
