"""Batched FEC framing on the GPU (include/rsmi_fec.h).

UDPspeeder's ``fec_encode_manager_t`` (fec_manager.cpp:174-460) turns a
connection's packets into FEC groups: mode 0 packs them into a length-prefixed
blob cut into k shards, mode 1 sends each packet as one zero-padded shard;
every packet gets the 8-byte header ``seq | mode | k | m | index`` and parity
comes from rs_encode2.  :class:`FecEncoder` holds one manager's state; a batch
of ``input()`` calls is planned on the host (lengths only) and framed, encoded
and carried over on the GPU:

    enc = FecEncoder("20:10", mode=0, mtu=1250, queue_len=200, seq0=1)
    plan = enc.plan(lens, offsets, in_buf)          # host lists, device input
    slots = torch.empty(plan.n_slots * S, dtype=torch.uint8, device="cuda")
    enc.run(slots, S)                                # frame + encode + carry
    for slot, length, event in plan.packets: ...     # output() order

``input`` / ``output`` keep the reference's per-call interface (one GPU batch
per call) for callers and tests that think in single packets.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from ._lib import check, lib, rsmi_fec_config, rsmi_fenc_packet

HEADER = 8
SLOT_PACKET = 120   # RSMI_FEC_SLOT_PACKET: packet offset in a slot
COOK_LEAD = SLOT_PACKET % 16  # RSMI_FEC_COOK_LEAD: first packet's offset in a packed cooked output
SLOT_SHARD = 128    # RSMI_FEC_SLOT_SHARD: shard offset (128-byte aligned rows)


def fec_config(rs_str: str, mode: int = 0, mtu: int = 1250, queue_len: int = 200,
               short_packet_optimize: int = 1, header_overhead: int = 40) -> rsmi_fec_config:
    """fec_parameter_t from a -f string (rs_from_str, fec_manager.h:40-136)."""
    cfg = rsmi_fec_config()
    check(lib().rsmi_fec_config_init(C.byref(cfg), rs_str.encode(), mode, mtu, queue_len),
          "rsmi_fec_config_init")
    cfg.short_packet_optimize = short_packet_optimize
    cfg.header_overhead = header_overhead
    return cfg


@dataclass
class FencPlan:
    n_slots: int
    slot_stride_min: int
    ret: np.ndarray          # input() return value per event
    packets: np.ndarray      # structured: slot, len, event (output() order)
    groups: dict             # slot0, k, m, fec_len, seq per completed group


class FecEncoder:
    """One fec_encode_manager_t; its device state lives on the current device."""

    def __init__(self, rs_str: str = "20:10", mode: int = 0, mtu: int = 1250,
                 queue_len: int = 200, seq0: int = 0, **kw):
        self.cfg = fec_config(rs_str, mode, mtu, queue_len, **kw)
        h = C.c_void_p()
        check(lib().rsmi_fenc_create(C.byref(self.cfg), C.c_uint32(seq0 & 0xFFFFFFFF), C.byref(h)),
              "rsmi_fenc_create")
        self._h = h
        self._keep = None

    def close(self):
        if getattr(self, "_h", None):
            lib().rsmi_fenc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_config(self, rs_str: str, mode: int = 0, mtu: int = 1250, queue_len: int = 200):
        """g_fec_par update: taken up at the next group start (fec_manager.cpp:207-209)."""
        cfg = fec_config(rs_str, mode, mtu, queue_len)
        check(lib().rsmi_fenc_next_config(self._h, C.byref(cfg)), "rsmi_fenc_next_config")

    def plan(self, lens, offsets=None, in_buf=None) -> FencPlan:
        """Plan input() for every event: lens[i] >= 0 is a packet of that many
        bytes at in_buf + offsets[i] (in_buf: CUDA uint8 tensor with 16 spare
        bytes after every packet), lens[i] < 0 is the timer flush input(0, 0)."""
        lens = np.ascontiguousarray(lens, np.int32)
        n = len(lens)
        offp = basep = None
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, np.uint64)
            offp = offsets.ctypes.data
        if isinstance(in_buf, int):
            basep = in_buf or None
        elif in_buf is not None:
            basep = in_buf.data_ptr()
        ret = np.zeros(n, np.int32)
        ns, npk, smin = C.c_int64(), C.c_int64(), C.c_int32()
        check(lib().rsmi_fenc_plan(self._h, n, lens.ctypes.data if n else None, offp, basep,
                                   ret.ctypes.data if n else None, C.byref(ns), C.byref(npk),
                                   C.byref(smin)), "rsmi_fenc_plan")
        pk = (rsmi_fenc_packet * max(1, npk.value))()
        check(lib().rsmi_fenc_packets(self._h, pk), "rsmi_fenc_packets")
        dt = np.dtype([("slot", np.int64), ("len", np.int32), ("event", np.int32)])
        packets = np.frombuffer(bytes(pk), dt)[:npk.value].copy()
        ng = C.c_int64()
        check(lib().rsmi_fenc_groups(self._h, C.byref(ng), None, None, None, None, None),
              "rsmi_fenc_groups")
        g = {"slot0": np.zeros(ng.value, np.int64), "k": np.zeros(ng.value, np.int32),
             "m": np.zeros(ng.value, np.int32), "fec_len": np.zeros(ng.value, np.int32),
             "seq": np.zeros(ng.value, np.uint32)}
        if ng.value:
            check(lib().rsmi_fenc_groups(self._h, None, g["slot0"].ctypes.data, g["k"].ctypes.data,
                                         g["m"].ctypes.data, g["fec_len"].ctypes.data,
                                         g["seq"].ctypes.data), "rsmi_fenc_groups")
        # the input must outlive the run, which may overlap the next plan
        self._keep = (in_buf, (self._keep or (None,))[0])
        self._last_packets = packets
        self._last_nslots = ns.value
        self._last_smin = smin.value
        self._last_npk = npk.value
        return FencPlan(ns.value, smin.value, ret, packets, g)

    def _check_slots(self, buf, slot_stride: int, what: str):
        """The kernels write at slot * slot_stride (+ the packet or shard
        offset) with no bound of their own: a buffer shorter than the last
        plan's n_slots * slot_stride would be written past its end."""
        need = getattr(self, "_last_nslots", 0) * int(slot_stride)
        if buf.numel() < need:
            raise ValueError(f"{what} holds {buf.numel()} bytes; the last plan needs "
                             f"n_slots * slot_stride = {need}")

    def plan_host(self, lens, offsets) -> FencPlan:
        """Plan only (no device): decisions, packet list and groups for a batch
        whose payloads are never framed -- for inspecting the schedule."""
        return self.plan(lens, offsets, 0)

    def run(self, slots, slot_stride: int, stream=None):
        """Frame + encode + carry the planned batch into `slots` (CUDA uint8,
        >= n_slots * slot_stride bytes); asynchronous on `stream`."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        self._check_slots(slots, slot_stride, "slots")
        check(lib().rsmi_fenc_run_dev(self._h, slots.data_ptr() if slots.numel() else None,
                                      int(slot_stride), s.cuda_stream), "rsmi_fenc_run_dev")

    def run_cooked(self, slots, slot_stride: int, cook, seed: int, out=None, out_len=None,
                   stream=None):
        """Frame + encode + carry the planned batch into `slots`, then do_cook
        every packet it emits into `out` at the same slot layout (None: in place
        in slots) -- rsmi_fenc_run_cooked_dev.  out may be pinned host memory:
        the cooked packets then reach the host in the cook kernel's own stores.
        cook: a cook.CookContext.  Returns the int32 CUDA tensor of cooked
        lengths, one per planned packet (-1: did not fit)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        npk = getattr(self, "_last_npk", None)
        if out_len is None:
            out_len = torch.empty(max(npk or 0, 1), dtype=torch.int32, device="cuda")
        elif out_len.dtype != torch.int32 or not out_len.is_cuda or out_len.numel() < (npk or 0):
            raise ValueError(f"out_len must be an int32 CUDA tensor of >= {npk} entries "
                             "(one per planned packet)")
        self._check_slots(slots, slot_stride, "slots")
        if out is not None:
            if out.dtype != torch.uint8 or not (out.is_cuda or out.is_pinned()) or out.data_ptr() % 16:
                raise TypeError("out must be a 16-aligned CUDA or pinned uint8 tensor")
            self._check_slots(out, slot_stride, "out")
        check(lib().rsmi_fenc_run_cooked_dev(self._h, slots.data_ptr() if slots.numel() else None,
                                             int(slot_stride), cook._h, C.c_uint64(seed & (2**64 - 1)),
                                             out.data_ptr() if out is not None else None,
                                             out_len.data_ptr(), s.cuda_stream),
              "rsmi_fenc_run_cooked_dev")
        return out_len

    def last_parity_cooked(self) -> int:
        """Encoder runs of the last cooked run whose parity packets were cooked
        in the encoder's epilogue (RSMI_OPT_PARITY_COOK) --
        rsmi_fenc_last_parity_cooked."""
        return int(lib().rsmi_fenc_last_parity_cooked(self._h))

    RUN_DTYPE = np.dtype([("slot", np.int64), ("out0", np.int64), ("first", np.int32),
                          ("afirst", np.int32), ("bfirst", np.int32), ("len", np.int32),
                          ("job", np.int32), ("count", np.uint16), ("ndata", np.uint16),
                          ("nfr", np.uint16), ("pad", np.uint16)],
                         align=True)  # 48 B, as in C

    def packet_runs(self) -> np.ndarray:
        """The last plan's packet list as runs (rsmi_fenc_packet_runs): what a
        cooked run uploads and expands on the device into its two cook lists."""
        n = C.c_int64()
        check(lib().rsmi_fenc_packet_runs(self._h, C.byref(n), None), "rsmi_fenc_packet_runs")
        assert self.RUN_DTYPE.itemsize == 48
        out = np.zeros(n.value, self.RUN_DTYPE)
        if n.value:
            check(lib().rsmi_fenc_packet_runs(self._h, C.byref(n), out.ctypes.data),
                  "rsmi_fenc_packet_runs")
        return out

    @staticmethod
    def cook_span(lens):
        """RSMI_FEC_COOK_SPAN: bytes a packet of len bytes takes in a packed
        cooked output (COOK_LEAD scratch bytes, then its cooked form, rounded
        up to 16-byte pieces)."""
        return (np.asarray(lens, np.int64) + 37 + COOK_LEAD + 15) // 16 * 16

    def packed_offsets(self):
        """Where run_cooked_packed puts each packet of the last plan, and the
        total bytes: (int64 offsets, total)."""
        sp = self.cook_span(self._last_packets["len"])
        offs = np.full(len(sp), COOK_LEAD, np.int64)
        if len(sp) > 1:
            offs[1:] += np.cumsum(sp[:-1])
        return offs, int(sp.sum())

    def run_cooked_packed(self, slots, slot_stride: int, cook, seed: int, out, out_len=None,
                          stream=None):
        """run_cooked with the cooked packets back to back in `out` (CUDA or
        pinned uint8, 16-aligned): packet p at packed_offsets()[0][p] --
        rsmi_fenc_run_cooked_packed_dev.  Returns the int32 CUDA tensor of
        cooked lengths."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        npk = len(self._last_packets)
        if out_len is None:
            out_len = torch.empty(max(npk, 1), dtype=torch.int32, device="cuda")
        elif out_len.dtype != torch.int32 or not out_len.is_cuda or out_len.numel() < npk:
            raise ValueError(f"out_len must be an int32 CUDA tensor of >= {npk} entries")
        self._check_slots(slots, slot_stride, "slots")
        if out.dtype != torch.uint8 or not (out.is_cuda or out.is_pinned()) or out.data_ptr() % 16:
            raise TypeError("out must be a 16-aligned CUDA or pinned uint8 tensor")
        check(lib().rsmi_fenc_run_cooked_packed_dev(
            self._h, slots.data_ptr() if slots.numel() else None, int(slot_stride), cook._h,
            C.c_uint64(seed & (2**64 - 1)), out.data_ptr(), int(out.numel()), out_len.data_ptr(),
            s.cuda_stream), "rsmi_fenc_run_cooked_packed_dev")
        return out_len

    def packets_now(self):
        """The last plan's packet list as it stands now (after
        FecCollector.run_many: slots of the shared slot array)."""
        npk = self._last_npk
        pk = (rsmi_fenc_packet * max(1, npk))()
        check(lib().rsmi_fenc_packets(self._h, pk), "rsmi_fenc_packets")
        dt = np.dtype([("slot", np.int64), ("len", np.int32), ("event", np.int32)])
        return np.frombuffer(bytes(pk), dt)[:npk].copy()

    @staticmethod
    def slot_stride_for(fec_len_max: int) -> int:
        """A multiple of 128 that fits fec_len_max-byte shards and do_cook's
        tail (rsmi_cook.h) in place: SLOT_SHARD + round_up(fec_len_max + 37, 128)."""
        return SLOT_SHARD + (fec_len_max + 37 + 127) // 128 * 128

    # ---- the reference's per-call interface (one GPU batch per call) ---------
    def input(self, data: Optional[bytes]) -> int:
        """fec_encode_manager_t::input(s, len); data None is input(0, 0)."""
        import torch
        if data is None:
            p = self.plan([-1])
            buf = torch.zeros(16, dtype=torch.uint8, device="cuda")
        else:
            buf = torch.zeros(len(data) + 16, dtype=torch.uint8)
            buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else buf[:0]
            buf = buf.cuda()
            p = self.plan([len(data)], [0], buf)
        stride = p.slot_stride_min
        slots = torch.zeros(max(1, p.n_slots) * stride, dtype=torch.uint8, device="cuda")
        self.run(slots, stride)
        host = slots.cpu().numpy()
        self._ready = [host[s * stride + SLOT_PACKET:s * stride + SLOT_PACKET + ln].tobytes()
                       for s, ln, _ in p.packets]
        return int(p.ret[0])

    def output(self) -> List[bytes]:
        """fec_encode_manager_t::output: the packets the last input() produced."""
        r, self._ready = getattr(self, "_ready", []), []
        return r


def packets_bytes(plan: FencPlan, slots_host: np.ndarray, slot_stride: int) -> List[bytes]:
    """The emitted packets of a run, as bytes (slots_host: the slot array on the host)."""
    return [slots_host[s * slot_stride + SLOT_PACKET:s * slot_stride + SLOT_PACKET + ln].tobytes()
            for s, ln, _ in plan.packets]


@dataclass
class FdecPlan:
    ret: np.ndarray      # input() return value per packet
    n_decodes: int       # groups the batch decodes


class FecDecoder:
    """One fec_decode_manager_t (fec_manager.cpp:469-797): received packets in,
    the packets output() returns out.  Decodes run batched on the GPU."""

    def __init__(self, buff_num: int = 0):
        h = C.c_void_p()
        check(lib().rsmi_fdec_create(int(buff_num), C.byref(h)), "rsmi_fdec_create")
        self._h = h
        self._keep = None

    def close(self):
        if getattr(self, "_h", None):
            lib().rsmi_fdec_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, host_buf: np.ndarray, lens, offsets, dev_buf=None, now_ms: int = 0) -> FdecPlan:
        """Plan input() for every packet: packet i is lens[i] bytes at
        host_buf[offsets[i]:] (host uint8 array) and at the same offset of
        dev_buf (CUDA uint8 tensor with the same bytes, 16 spare after each)."""
        lens = np.ascontiguousarray(lens, np.int32)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(lens)
        ret = np.zeros(n, np.int32)
        nd = C.c_int64()
        devp = dev_buf.data_ptr() if dev_buf is not None else None  # None: plan only
        check(lib().rsmi_fdec_plan(self._h, n, lens.ctypes.data, offsets.ctypes.data,
                                   host_buf.ctypes.data, devp, int(now_ms), ret.ctypes.data,
                                   C.byref(nd)), "rsmi_fdec_plan")
        # batch i's buffers stay referenced while batch i+1 is planned and run
        self._keep = ((host_buf, dev_buf), (self._keep or (None,))[0])
        return FdecPlan(ret, nd.value)

    def run(self, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        check(lib().rsmi_fdec_run_dev(self._h, s.cuda_stream), "rsmi_fdec_run_dev")

    def outputs_raw(self):
        """(ptr, len, event) arrays of the outputs, in output() order, without
        copying the bytes (waits for the run; pointers live until the next plan)."""
        n = C.c_int64()
        check(lib().rsmi_fdec_outputs(self._h, C.byref(n)), "rsmi_fdec_outputs")
        ptr = np.zeros(max(1, n.value), np.uint64)
        ln = np.zeros(max(1, n.value), np.int32)
        ev = np.zeros(max(1, n.value), np.int32)
        check(lib().rsmi_fdec_output_list(self._h, ptr.ctypes.data, ln.ctypes.data,
                                          ev.ctypes.data), "rsmi_fdec_output_list")
        return ptr[:n.value], ln[:n.value], ev[:n.value]

    def outputs(self):
        """[(bytes, event)] in the reference's output() order (waits for the run)."""
        ptr, ln, ev = self.outputs_raw()
        return [(C.string_at(int(ptr[i]), int(ln[i])) if ln[i] else b"", int(ev[i]))
                for i in range(len(ln))]

    # ---- the reference's per-call interface ------------------------------------
    def input(self, packet: bytes, now_ms: int = 0) -> int:
        """fec_decode_manager_t::input(s, len) for one packet (one GPU batch)."""
        import torch
        host = np.zeros(len(packet) + 16, np.uint8)
        host[:len(packet)] = np.frombuffer(bytes(packet), np.uint8)
        dev = torch.from_numpy(host).cuda()
        p = self.plan(host, [len(packet)], [0], dev, now_ms)
        self.run()
        self._ready = [b for b, _ in self.outputs()]
        return int(p.ret[0])

    def output(self) -> List[bytes]:
        """fec_decode_manager_t::output: the packets the last input() produced."""
        r, self._ready = getattr(self, "_ready", []), []
        return r


class FecCollector:
    """rsmi_fenc_run_many: many connections' encoders (each planned on its own
    state with FecEncoder.plan) run as one launch set over one slot array
    (include/rsmi_fec.h, "the collector").  After run_many each encoder's
    packets_now() lists its packets at slots of the shared array."""

    def __init__(self):
        h = C.c_void_p()
        check(lib().rsmi_fcol_create(C.byref(h)), "rsmi_fcol_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().rsmi_fcol_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan_many(self, encoders, lens, offsets, in_buf, nthreads: int = 8):
        """rsmi_fenc_plan_many: plan every encoder's batch (lens[i], offsets[i]
        into the one in_buf) on up to nthreads host threads.  Returns the
        per-encoder (n_slots, n_packets, slot_stride_min) arrays; the
        encoders' packet lists are read with packets_now() after the run."""
        n = len(encoders)
        counts = np.array([len(l) for l in lens], np.int64)
        ev0 = np.zeros(n + 1, np.int64)
        np.cumsum(counts, out=ev0[1:])
        L = np.ascontiguousarray(np.concatenate(lens) if n else np.zeros(0), np.int32)
        O = np.ascontiguousarray(np.concatenate(offsets) if n else np.zeros(0), np.uint64)
        ret = np.zeros(max(1, L.size), np.int32)
        ns = np.zeros(max(1, n), np.int64)
        npk = np.zeros(max(1, n), np.int64)
        smin = np.zeros(max(1, n), np.int32)
        arr = (C.c_void_p * max(1, n))(*[e._h.value for e in encoders])
        base = in_buf if isinstance(in_buf, int) else (in_buf.data_ptr() if in_buf is not None else None)
        check(lib().rsmi_fenc_plan_many(arr, n, ev0.ctypes.data, L.ctypes.data if L.size else None,
                                        O.ctypes.data if O.size else None, base or None, ret.ctypes.data,
                                        ns.ctypes.data, npk.ctypes.data, smin.ctypes.data, int(nthreads)),
              "rsmi_fenc_plan_many")
        for i, e in enumerate(encoders):
            e._last_nslots, e._last_npk, e._last_smin = int(ns[i]), int(npk[i]), int(smin[i])
            e._last_packets = None
            e._keep = (in_buf, (e._keep or (None,))[0])
        self.last_ret = ret[:L.size]
        return ns[:n], npk[:n], smin[:n]

    def run_many(self, encoders, slots, slot_stride: int, cook=None, seed: int = 0, out=None,
                 out_len=None, stream=None):
        """Frame + encode (+ do_cook into `out`, None: in place) every encoder's
        planned batch on `stream`.  slots: CUDA uint8 of >= sum(n_slots) *
        slot_stride bytes.  With cook, returns the int32 cooked lengths of all
        packets, the encoders' lists concatenated in order."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        n_slots = sum(e._last_nslots for e in encoders)
        n_pk = sum(e._last_npk for e in encoders)
        smin = max((getattr(e, "_last_smin", 0) for e in encoders), default=0)
        if int(slot_stride) % 16 or int(slot_stride) < smin:
            raise ValueError(f"slot_stride must be a multiple of 16 >= every encoder's slot_stride_min ({smin})")
        if slots.numel() < n_slots * int(slot_stride):
            raise ValueError(f"slots holds {slots.numel()} bytes; the encoders need {n_slots * slot_stride}")
        if cook is not None and out_len is None:
            out_len = torch.empty(max(n_pk, 1), dtype=torch.int32, device="cuda")
        elif out_len is not None and (out_len.dtype != torch.int32 or not out_len.is_cuda
                                      or out_len.numel() < n_pk):
            # the cook writes out_len[i] for the whole concatenated packet list
            raise ValueError(f"out_len must be an int32 CUDA tensor of >= {n_pk} entries "
                             "(one per planned packet of every encoder)")
        if out is not None:
            if out.dtype != torch.uint8 or not (out.is_cuda or out.is_pinned()) or out.data_ptr() % 16:
                raise TypeError("out must be a 16-aligned CUDA or pinned uint8 tensor")
            if out.numel() < n_slots * int(slot_stride):
                raise ValueError("out is shorter than the shared slot array")
        arr = (C.c_void_p * max(1, len(encoders)))(*[e._h.value for e in encoders])
        check(lib().rsmi_fenc_run_many(self._h, arr, len(encoders),
                                       slots.data_ptr() if slots.numel() else None, int(slot_stride),
                                       cook._h if cook is not None else None, C.c_uint64(seed & (2**64 - 1)),
                                       out.data_ptr() if out is not None else None,
                                       out_len.data_ptr() if out_len is not None else None, s.cuda_stream),
              "rsmi_fenc_run_many")
        return out_len


class FecDecodeCollector:
    """rsmi_fdec_run_many: many connections' decoders (each planned on its own
    state with FecDecoder.plan) run as one launch set; afterwards each
    decoder's outputs() works as after its own run()."""

    def __init__(self):
        h = C.c_void_p()
        check(lib().rsmi_fdcol_create(C.byref(h)), "rsmi_fdcol_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().rsmi_fdcol_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan_many(self, decoders, host_bufs, lens, offsets, dev_bufs=None, now_ms: int = 0,
                  nthreads: int = 8):
        """rsmi_fdec_plan_many: FecDecoder.plan for every decoder (packets
        lens[i] / offsets[i] into host_bufs[i] and dev_bufs[i]; dev_bufs None:
        plan only) on up to nthreads host threads.  Returns the per-decoder
        FdecPlan list."""
        n = len(decoders)
        counts = np.array([len(l) for l in lens], np.int64)
        pk0 = np.zeros(n + 1, np.int64)
        np.cumsum(counts, out=pk0[1:])
        L = np.ascontiguousarray(np.concatenate(lens) if n else np.zeros(0), np.int32)
        O = np.ascontiguousarray(np.concatenate(offsets) if n else np.zeros(0), np.uint64)
        ret = np.zeros(max(1, L.size), np.int32)
        nd = np.zeros(max(1, n), np.int64)
        arr = (C.c_void_p * max(1, n))(*[d._h.value for d in decoders])
        hb = (C.c_void_p * max(1, n))(*[h.ctypes.data for h in host_bufs])
        db = None
        if dev_bufs is not None:
            db = (C.c_void_p * max(1, n))(*[(d.data_ptr() if d is not None else None) for d in dev_bufs])
        check(lib().rsmi_fdec_plan_many(arr, n, pk0.ctypes.data, L.ctypes.data if L.size else None,
                                        O.ctypes.data if O.size else None, hb, db, int(now_ms),
                                        ret.ctypes.data, nd.ctypes.data, int(nthreads)), "rsmi_fdec_plan_many")
        plans = []
        for i, d in enumerate(decoders):
            dv = dev_bufs[i] if dev_bufs is not None else None
            d._keep = ((host_bufs[i], dv), (d._keep or (None,))[0])
            plans.append(FdecPlan(ret[pk0[i]:pk0[i + 1]].copy(), int(nd[i])))
        return plans

    def run_many(self, decoders, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        arr = (C.c_void_p * max(1, len(decoders)))(*[d._h.value for d in decoders])
        check(lib().rsmi_fdec_run_many(self._h, arr, len(decoders), s.cuda_stream), "rsmi_fdec_run_many")
