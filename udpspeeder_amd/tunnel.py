"""The tunnel's data path, batched (SURVEY §8f f4 with f1-f3): UDP datagrams
in, FEC framing + encode + cook on the GPU, UDP datagrams out -- and the
reverse.  One step moves one batch; a connection owns one Sender and one
Receiver.  This is the per-packet loop of the reference --

* send side, tunnel_client.cpp:41-80 (local_listen_cb): recvfrom one datagram,
  from_normal_to_fec (fec_encode_manager_t::input/output), my_send each
  output packet (do_cook + sendto, packet.cpp:165-168);
* receive side, tunnel_client.cpp:110-160 (remote_cb): recv one datagram,
  de_cook, from_fec_to_normal (fec_decode_manager_t::input/output), sendto
  each output --

with the sockets read and written by recvmmsg / sendmmsg (udpspeeder_amd.io),
the managers by rsmi_fenc_* / rsmi_fdec_*, and cook / de_cook by their GPU
kernels.  The conv-id layer (get_conv / put_conv, connection.h) that
multiplexes UDP flows inside one tunnel is not part of this path.
"""
import numpy as np

from . import io
from .cook import CookContext
from .fec import SLOT_PACKET, FecDecoder, FecEncoder


def _round_up(x, a):
    return (x + a - 1) // a * a


class _View:
    """(ptr, stride) of a pinned torch tensor, for io.recv_batch / send_batch."""

    def __init__(self, t, stride):
        self.ptr = t.data_ptr()
        self.stride = stride


class Sender:
    """Datagrams from the local application -> FEC groups -> cooked packets out."""

    def __init__(self, rs: str = "20:10", mode: int = 0, mtu: int = 1250, queue_len: int = 200,
                 key: bytes = b"", batch: int = 32768, max_len: int = 1400, seq0: int = 1,
                 stream=None):
        import torch
        self.torch = torch
        self.enc = FecEncoder(rs, mode, mtu, queue_len, seq0=seq0)
        self.cook = CookContext(key)
        self.batch, self.max_len = batch, max_len
        self.sin = _round_up(max_len + 1 + 16, 128)         # input slot: datagram + 16 spare
        self.s = FecEncoder.slot_stride_for(max(mtu, max_len + 2))  # output slot (fec_len <= it)
        self.stream = stream or torch.cuda.Stream()
        self.h_in = torch.empty(batch * self.sin, dtype=torch.uint8).pin_memory()
        self.d_in = torch.empty(batch * self.sin, dtype=torch.uint8, device="cuda")
        self.slots = None
        self.d_out = self.h_out = None
        self.seed = seq0

    def _emit(self, p, sock_out, to, drop):
        """Frame + encode + cook the planned batch in one run
        (rsmi_fenc_run_cooked_packed_dev): the cooked packets land back to back
        in device memory, and only those bytes cross PCIe for sendmmsg."""
        torch = self.torch
        S = self.s
        if p.n_slots == 0 or len(p.packets) == 0:
            return 0
        offs, total = self.enc.packed_offsets()
        if self.slots is None or self.slots.numel() < p.n_slots * S:
            self.slots = torch.empty(p.n_slots * S, dtype=torch.uint8, device="cuda")
        if self.d_out is None or self.d_out.numel() < total:
            self.d_out = torch.empty(total, dtype=torch.uint8, device="cuda")
            self.h_out = torch.empty(total, dtype=torch.uint8).pin_memory()
        with torch.cuda.stream(self.stream):
            self.seed += 1
            out_len = self.enc.run_cooked_packed(self.slots, S, self.cook, self.seed, self.d_out,
                                                 stream=self.stream)
            self.h_out[:total].copy_(self.d_out[:total], non_blocking=True)
            ol = out_len.to("cpu", non_blocking=True)
        self.stream.synchronize()
        ol = ol.numpy()[:len(p.packets)].copy()
        if drop is not None:
            ol[drop(p)] = -1  # lost on the way (tests / benches)
        keep = ol >= 0
        ptrs = (offs + self.h_out.data_ptr()).astype(np.uint64)
        return io.send_ptrs(sock_out, ptrs[keep], ol[keep], to)

    def step(self, sock_in, sock_out, to, timeout_ms: int = 50, drop=None):
        """One batch: returns (datagrams read, packets sent)."""
        torch = self.torch
        lens = io.recv_batch(sock_in, _View(self.h_in, self.sin), 0, self.max_len, self.batch,
                             timeout_ms)
        n = len(lens)
        if n == 0:
            return 0, 0
        keep = np.nonzero(lens >= 0)[0]  # longer than max_len: dropped (tunnel_client.cpp:50-53)
        with torch.cuda.stream(self.stream):
            self.d_in[:n * self.sin].copy_(self.h_in[:n * self.sin], non_blocking=True)
        self.stream.synchronize()  # the plan's device addresses point into d_in
        p = self.enc.plan(lens[keep], keep.astype(np.uint64) * np.uint64(self.sin), self.d_in)
        return n, self._emit(p, sock_out, to, drop)

    def flush(self, sock_out, to, drop=None):
        """The FEC timer (input(0, 0), tunnel_client.cpp:41): close the open group."""
        p = self.enc.plan(np.array([-1], np.int32), np.zeros(1, np.uint64), self.d_in)
        return self._emit(p, sock_out, to, drop)


class Receiver:
    """Cooked packets in -> de_cook -> FEC decode -> datagrams to the application."""

    def __init__(self, key: bytes = b"", batch: int = 65536, max_len: int = 1500, stream=None):
        import torch
        self.torch = torch
        self.dec = FecDecoder()
        self.cook = CookContext(key)
        self.batch, self.max_len = batch, max_len
        self.s = _round_up(max_len + 1 + 16, 128)
        self.stream = stream or torch.cuda.Stream()
        self.h = torch.empty(batch * self.s, dtype=torch.uint8).pin_memory()
        self.d = torch.empty(batch * self.s, dtype=torch.uint8, device="cuda")
        self.host = self.h.numpy()

    def step(self, sock_in, sock_out, to, timeout_ms: int = 50, now_ms: int = 0):
        """One batch: returns (packets read, datagrams delivered)."""
        torch = self.torch
        S = self.s
        lens = io.recv_batch(sock_in, _View(self.h, S), 0, self.max_len, self.batch, timeout_ms)
        n = len(lens)
        if n == 0:
            return 0, 0
        with torch.cuda.stream(self.stream):
            self.d[:n * S].copy_(self.h[:n * S], non_blocking=True)
            lt = torch.from_numpy(np.maximum(lens, 0).astype(np.int32)).to("cuda", non_blocking=True)
            # de_cook in place on the device (the FEC gather reads it there) and
            # into the pinned receive buffer (the planner reads headers and the
            # outputs point into it): only packet bytes come back over PCIe
            out_len = self.cook.decook_mirror(self.d[:n * S], lt, self.h, cap=S, stride=S,
                                              stream=self.stream)
            ol = out_len.to("cpu", non_blocking=True)
        self.stream.synchronize()
        ol = ol.numpy().copy()
        ol[lens < 0] = -1
        offs_h = np.arange(n, dtype=np.uint64) * np.uint64(S)
        self.dec.plan(self.host, ol, offs_h, self.d, now_ms=now_ms)
        self.dec.run(stream=self.stream)
        ptr, ln, _ = self.dec.outputs_raw()
        return n, io.send_ptrs(sock_out, ptr, ln, to)
