"""FEC framing: fec_encode_manager_t batched on the GPU.

CPU tests pin the Python restatement (oracle/fec_frame.py) to the fixtures the
REAL reference manager produced (tests/golden/fec_encode.npz, written by
oracle/gen_golden_fec.py), and check librsmi.so's host planner -- return codes,
packet lengths, output() order, group boundaries -- against them without a GPU.
GPU tests frame + encode through the C ABI and compare every packet byte with
the fixtures and, at larger sizes, with the restatement; batches are cut at
arbitrary event boundaries so groups straddle batches (the carry area).
"""
import hashlib
import os

import numpy as np
import pytest

from oracle.cpu import cook_payloads
from oracle.fec_frame import EncodeManager
from oracle.gen_golden_fec import CASES, case_events

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fec_encode.npz")


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(GOLDEN))


def _case(fx, name):
    ci = [c[0] for c in CASES].index(name)
    _, rs, mode, mtu, ql, n, lmax, fpm, zpm = CASES[ci]
    lens, ev = case_events(ci, n, lmax, fpm, zpm)
    assert (lens == fx[f"{name}__lens"]).all()
    meta = fx[f"{name}__meta"]
    return dict(rs=rs, mode=mode, mtu=mtu, ql=ql, lens=lens, ev=ev, seq0=int(meta[4]),
                ret=fx[f"{name}__ret"], pk_len=fx[f"{name}__pk_len"],
                pk_event=fx[f"{name}__pk_event"], sha=fx[f"{name}__sha256"].tobytes(),
                full=fx.get(f"{name}__pk_bytes"))


def _expected_packets(c):
    if c["full"] is None:
        return None
    off = np.concatenate([[0], np.cumsum(c["pk_len"])])
    b = c["full"].tobytes()
    return [b[off[i]:off[i + 1]] for i in range(len(c["pk_len"]))]


NAMES = [c[0] for c in CASES]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_fixtures(fx, name):
    c = _case(fx, name)
    em = EncodeManager(c["rs"], c["mode"], c["mtu"], c["ql"], c["seq0"])
    ret, pk, pev = [], [], []
    for i, e in enumerate(c["ev"]):
        ret.append(em.input(e))
        o = em.output()
        pk += o
        pev += [i] * len(o)
    assert ret == list(c["ret"])
    assert pev == list(c["pk_event"])
    assert [len(p) for p in pk] == list(c["pk_len"])
    assert hashlib.sha256(b"".join(pk)).digest() == c["sha"]
    exp = _expected_packets(c)
    if exp is not None:
        assert pk == exp


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("nbatch", [1, 3])
def test_planner_matches_reference_fixtures(fx, name, nbatch):
    """librsmi.so's planner (no GPU): ret, packet lengths and events, group headers."""
    from udpspeeder_amd.fec import FecEncoder
    c = _case(fx, name)
    enc = FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"])
    lens = c["lens"]
    cuts = np.linspace(0, len(lens), nbatch + 1).astype(int)
    ret, plen, pev, nslot = [], [], [], 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        offs = np.zeros(b - a, np.uint64)
        p = enc.plan_host(lens[a:b], offs)
        ret += list(p.ret)
        plen += list(p.packets["len"])
        pev += list(p.packets["event"] + a)
        assert (p.packets["slot"] >= 0).all() and (p.packets["slot"] < p.n_slots).all()
        nslot += p.n_slots
    assert ret == list(c["ret"])
    assert plen == list(c["pk_len"])
    assert pev == list(c["pk_event"])
    enc.close()


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("nbatch", [1, 3])
def test_packet_runs_expand_to_the_packet_list(fx, name, nbatch):
    """The runs a cooked run uploads (no GPU): expanded as k_expand_packets
    does, they give every packet of rsmi_fenc_packets once, in order, with its
    slot and length.  In a fused run, list A (the data shards the fused
    framing cook frames: a mode-0 group's leading ones, every mode-1 data
    packet) and list B (every packet it does not cook, every parity packet)
    each keep packet order, and every packet is cooked once: from A if it is
    among its run's first ndata, else from B."""
    from udpspeeder_amd.fec import FecEncoder
    c = _case(fx, name)
    enc = FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"])
    lens = c["lens"]
    cuts = np.linspace(0, len(lens), nbatch + 1).astype(int)
    for a, b in zip(cuts[:-1], cuts[1:]):
        p = enc.plan_host(lens[a:b], np.zeros(b - a, np.uint64))
        runs = enc.packet_runs()
        npk = len(p.packets)
        slot, ln = np.full(npk, -1, np.int64), np.full(npk, -1, np.int64)
        la, lb, cooked = [], [], []
        for r in runs:
            assert int(r["ndata"]) <= int(r["nfr"]) <= int(r["count"])
            for c_ in range(int(r["count"])):
                i = int(r["first"]) + c_
                assert slot[i] == -1, "packet listed twice"
                slot[i], ln[i] = int(r["slot"]) + c_, int(r["len"])
                if c_ < int(r["nfr"]):
                    la.append((int(r["afirst"]) + c_, i))
                if c_ >= int(r["ndata"]):
                    lb.append((int(r["bfirst"]) + c_ - int(r["ndata"]), i))
                cooked.append(i)
        assert sorted(cooked) == list(range(npk))
        assert (slot == p.packets["slot"]).all() and (ln == p.packets["len"]).all()
        for lst in (la, lb):
            lst.sort()
            assert [x for x, _ in lst] == list(range(len(lst)))
            assert [i for _, i in lst] == sorted(i for _, i in lst)
        # list A holds data packets only (a run's leading data packets),
        # every parity packet is in list B
        g = p.groups
        kind = {}
        for s0, k, m in zip(g["slot0"], g["k"], g["m"]):
            for j in range(int(k) + int(m)):
                kind[int(s0) + j] = j >= int(k)
        par = {i for _, i in lb}
        for i in range(npk):
            if kind.get(int(p.packets["slot"][i]), False):
                assert i in par, i
        assert not any(kind.get(int(p.packets["slot"][i]), False) for _, i in la)
        if c["mode"] == 1:  # mode-1 data shards are always clean
            assert all(not kind.get(int(p.packets["slot"][i]), False) for _, i in la)
            assert len(la) == sum(1 for i in range(npk) if not kind.get(int(p.packets["slot"][i]), False))
    enc.close()


@pytest.mark.gpu
def test_gpu_packed_cook_bounds(gpu):
    """rsmi_fenc_run_cooked_packed_dev refuses an out_cap one byte short of the
    packed spans, before any launch; with the exact size every packet fits and
    sits RSMI_FEC_COOK_LEAD bytes into its 16-aligned span."""
    import torch
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import COOK_LEAD, FecEncoder
    enc = FecEncoder("20:10", 0, 1250, 200, seq0=3)
    ctx = CookContext(b"k")
    lens = np.array([1000, 17, 0, 1200, 64, -1], np.int32)
    offs = np.array([0, 1008, 1040, 1056, 2272, 0], np.uint64)
    inbuf = torch.randint(0, 256, (4096,), dtype=torch.uint8, device="cuda")
    p = enc.plan(lens, offs, inbuf)
    S = p.slot_stride_min
    slots = torch.zeros(p.n_slots * S, dtype=torch.uint8, device="cuda")
    po, total = enc.packed_offsets()
    assert total % 16 == 0 and (po % 16 == COOK_LEAD).all()
    short = torch.zeros(total, dtype=torch.uint8, device="cuda")
    with pytest.raises(Exception, match="out_cap"):
        enc.run_cooked_packed(slots, S, ctx, 1, short[:total - 16])
    ol = enc.run_cooked_packed(slots, S, ctx, 1, short).cpu().numpy()[:len(p.packets)]
    assert (ol >= p.packets["len"] + 9).all()
    assert (po + ol <= np.append(po[1:] - COOK_LEAD, total)).all()
    enc.close()
    ctx.close()


def _run_gpu(enc, lens, ev, cuts, torch):
    """Run the events through the GPU in batches; returns the emitted packets."""
    out = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        ln = lens[a:b]
        offs = np.zeros(b - a, np.uint64)
        o = 0
        chunks = []
        for i in range(a, b):
            offs[i - a] = o
            if ev[i] is not None:
                chunks.append(ev[i])
                o += len(ev[i])
        host = np.frombuffer(b"".join(chunks) + bytes(32), np.uint8)
        inbuf = torch.from_numpy(host.copy()).cuda()
        p = enc.plan(ln, offs, inbuf)
        S = (p.slot_stride_min + 127) // 128 * 128
        slots = torch.full((max(1, p.n_slots) * S,), 0xEE, dtype=torch.uint8, device="cuda")
        enc.run(slots, S)
        h = slots.cpu().numpy()
        del inbuf  # the carry area holds what the next batch needs
        out += [(h[s * S + 120:s * S + 120 + l].tobytes(), int(e) + a) for s, l, e in p.packets]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("nbatch", [1, 4])
def test_gpu_frames_match_reference(fx, gpu, name, nbatch):
    import torch
    from udpspeeder_amd.fec import FecEncoder
    c = _case(fx, name)
    enc = FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"])
    rng = np.random.default_rng(len(name) * 7 + nbatch)
    n = len(c["lens"])
    cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n, nbatch - 1)])) if nbatch > 1 \
        else np.array([0, n])
    out = _run_gpu(enc, c["lens"], c["ev"], cuts, torch)
    pk = [p for p, _ in out]
    assert [e for _, e in out] == list(c["pk_event"])
    assert [len(p) for p in pk] == list(c["pk_len"])
    exp = _expected_packets(c)
    if exp is not None:
        bad = [i for i, (a, b) in enumerate(zip(pk, exp)) if a != b]
        assert not bad, (len(bad), bad[:5])
    assert hashlib.sha256(b"".join(pk)).digest() == c["sha"]
    enc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rs,mode,mtu,ql,lmax", [
    ("20:10", 0, 1250, 200, 1250), ("1:3,2:4,10:6,20:10", 0, 1250, 200, 700),
    ("20:10", 1, 1250, 200, 1250), ("10:5,40:20", 0, 1400, 200, 1400),
    ("1:3,2:4,10:6,20:10", 1, 1250, 200, 900)])
def test_gpu_frames_match_oracle_large(gpu, rs, mode, mtu, ql, lmax):
    """Thousands of groups per batch, several batches, against the restatement."""
    import torch
    from udpspeeder_amd.fec import FecEncoder
    rng = np.random.default_rng(mtu + lmax + mode)
    n = 12000
    lens = rng.integers(0, lmax + 1, n).astype(np.int32)
    lens[rng.random(n) < 0.01] = -1
    pay = cook_payloads(0xF00D + mode, 0, n, np.maximum(lens, 0), lmax)
    ev = [None if lens[i] < 0 else pay[i, :lens[i]].tobytes() for i in range(n)]
    enc = FecEncoder(rs, mode, mtu, ql, seq0=0xFFFFFFF0)
    em = EncodeManager(rs, mode, mtu, ql, 0xFFFFFFF0)
    exp = []
    for i, e in enumerate(ev):
        em.input(e)
        exp += [(p, i) for p in em.output()]
    out = _run_gpu(enc, lens, ev, np.array([0, 5000, 5001, n]), torch)
    assert len(out) == len(exp)
    bad = [i for i, (a, b) in enumerate(zip(out, exp)) if a != b]
    assert not bad, (len(bad), bad[:5])
    enc.close()


def _run_gpu_pipelined(enc, lens, ev, cuts, torch):
    """As _run_gpu, but batch i+1 is planned while batch i still runs, and the
    batches alternate between two streams (the double-buffered plan sets)."""
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    pending = []
    for bi, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        ln = lens[a:b]
        offs = np.zeros(b - a, np.uint64)
        o = 0
        chunks = []
        for i in range(a, b):
            offs[i - a] = o
            if ev[i] is not None:
                chunks.append(ev[i])
                o += len(ev[i])
        s = streams[bi % 2]
        with torch.cuda.stream(s):
            inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()
                                     ).to("cuda", non_blocking=False)
            p = enc.plan(ln, offs, inbuf)  # the previous batch may still be on the GPU
            S = (p.slot_stride_min + 127) // 128 * 128
            slots = torch.full((max(1, p.n_slots) * S,), 0xEE, dtype=torch.uint8, device="cuda")
            enc.run(slots, S, stream=s)
        pending.append((p, slots, S, inbuf, a))
    torch.cuda.synchronize()
    out = []
    for p, slots, S, _, a in pending:
        h = slots.cpu().numpy()
        out += [(h[s * S + 120:s * S + 120 + l].tobytes(), int(e) + a) for s, l, e in p.packets]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("rs,mode", [("20:10", 0), ("1:3,2:4,10:6,20:10", 1)])
def test_gpu_frames_pipelined_two_streams(gpu, rs, mode):
    """Planning batch i+1 during batch i's GPU run, on two streams, gives the
    restatement's packets byte for byte."""
    import torch
    from udpspeeder_amd.fec import FecEncoder
    rng = np.random.default_rng(41 + mode)
    n = 9000
    lens = rng.integers(0, 1000, n).astype(np.int32)
    lens[rng.random(n) < 0.01] = -1
    pay = cook_payloads(0xBEEF + mode, 0, n, np.maximum(lens, 0), 1000)
    ev = [None if lens[i] < 0 else pay[i, :lens[i]].tobytes() for i in range(n)]
    enc = FecEncoder(rs, mode, 1250, 200, seq0=5)
    em = EncodeManager(rs, mode, 1250, 200, 5)
    exp = []
    for i, e in enumerate(ev):
        em.input(e)
        exp += [(p, i) for p in em.output()]
    cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n, 7)]))
    out = _run_gpu_pipelined(enc, lens, ev, cuts, torch)
    assert len(out) == len(exp)
    bad = [i for i, (a, b) in enumerate(zip(out, exp)) if a != b]
    assert not bad, (len(bad), bad[:5])
    enc.close()


@pytest.mark.gpu
def test_gpu_per_call_interface(gpu):
    """input()/output() one event at a time, as fec_manager's callers use it
    (misc.cpp:401-411: three packets then the timer flush)."""
    from udpspeeder_amd.fec import FecEncoder
    enc = FecEncoder("20:10", 0, 1250, 200, seq0=77)
    em = EncodeManager("20:10", 0, 1250, 200, 77)
    for d in [b"11111", b"22", b"33333333", None, b"a" * 7, b"b" * 13, b"ccc", None]:
        assert enc.input(d) == em.input(d)
        assert enc.output() == em.output()
    enc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("nbatch,host,packed", [(1, True, False), (3, False, False), (2, False, True),
                                                (1, True, True)])
def test_gpu_frames_cooked_match_reference(fx, gpu, cook_oracle, name, nbatch, host, packed):
    """rsmi_fenc_run_cooked_dev: framing + encode + do_cook in one run, cooked
    packets written straight into pinned host memory (or another device
    buffer), in the slot layout or packed back to back
    (rsmi_fenc_run_cooked_packed_dev).  IVs are the device draw of (seed,
    packet index), so every cooked
    packet is checked byte for byte against the oracle's do_cook of the
    reference manager's packet (tests/golden/fec_encode.npz) where the fixture
    holds full bytes, and through the oracle's de_cook against the fixture's
    digest everywhere."""
    import torch
    from oracle.cpu import device_ivs
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecEncoder
    c = _case(fx, name)
    key = b"secret key"
    enc = FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"])
    ctx = CookContext(key)
    lens, ev = c["lens"], c["ev"]
    n = len(lens)
    cuts = np.linspace(0, n, nbatch + 1).astype(int)
    cooked, ivs = [], []
    for bi, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        offs = np.zeros(b - a, np.uint64)
        o, chunks = 0, []
        for i in range(a, b):
            offs[i - a] = o
            if ev[i] is not None:
                chunks.append(ev[i])
                o += len(ev[i])
        inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()).cuda()
        p = enc.plan(lens[a:b], offs, inbuf)
        # packed: the smallest legal stride (the packed output needs no tail room)
        S = p.slot_stride_min if packed else FecEncoder.slot_stride_for(max(p.slot_stride_min - 128, 0))
        slots = torch.full((max(1, p.n_slots) * S,), 0xEE, dtype=torch.uint8, device="cuda")
        if packed:
            po, ptot = enc.packed_offsets()
            out = torch.zeros(max(ptot, 16), dtype=torch.uint8)
        else:
            out = torch.zeros(max(1, p.n_slots) * S, dtype=torch.uint8)
        out = out.pin_memory() if host else out.cuda()
        seed = 1000 + bi
        if packed:
            ol = enc.run_cooked_packed(slots, S, ctx, seed, out)
        else:
            ol = enc.run_cooked(slots, S, ctx, seed, out=out)
        torch.cuda.synchronize()
        ol = ol.cpu().numpy()[:len(p.packets)]
        h = out.cpu().numpy()
        iv, ivl = device_ivs(seed, 0, len(p.packets))
        for i, (s, ln, _) in enumerate(p.packets):
            assert ol[i] == ln + 4 + ivl[i] + 1, (bi, i)
            o = int(po[i]) if packed else s * S + 120
            cooked.append(h[o:o + ol[i]].tobytes())
            ivs.append(iv[i, :ivl[i]].tobytes())
        del inbuf
    assert len(cooked) == len(c["pk_len"])
    plain = []
    for ck in cooked:
        rc, b, nl = cook_oracle.de_cook(ck, key)
        assert rc == 0
        plain.append(b[:nl])
    assert [len(p) for p in plain] == list(c["pk_len"])
    assert hashlib.sha256(b"".join(plain)).digest() == c["sha"]
    exp = _expected_packets(c)
    if exp is not None:
        bad = [i for i, (ck, e, v) in enumerate(zip(cooked, exp, ivs))
               if ck != cook_oracle.do_cook(e, v, key)]
        assert not bad, (len(bad), bad[:5])
    enc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cook,native_plan", [(False, False), (True, False), (True, True)])
def test_gpu_collector_200_connections_match_reference(fx, gpu, cook, native_plan, cook_oracle):
    """The cross-connection collector (rsmi_fenc_run_many): 200 managers --
    max_conn_num, common.h:112, one per connection (connection.h:244-245) --
    each fed its own golden event stream (case i % 10, cut into 3 batches at
    per-connection points, so groups straddle batches through each manager's
    carry area), planned one by one, run together per flush: every
    connection's packets equal the reference's (order, events, bytes).  With
    cook, the cooked packets are do_cook of those (the oracle, each with the
    IV the device drew), de_cook restores them."""
    import torch
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecCollector, FecEncoder
    ncon = 200
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(ncon)]
    encs = [FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"]) for c in cases]
    rng = np.random.default_rng(200)
    cuts = []
    col = FecCollector()
    for c in cases:
        n = len(c["lens"])
        a, b = sorted(rng.integers(1, n, 2))
        cuts.append([0, int(a), int(b), n])
    ctx = CookContext(b"collector-key") if cook else None
    got = [[] for _ in range(ncon)]
    for bi in range(3):
        chunks, offs_all, o = [], [], 0
        for ci, c in enumerate(cases):
            a, b = cuts[ci][bi], cuts[ci][bi + 1]
            offs = np.zeros(b - a, np.uint64)
            for i in range(a, b):
                offs[i - a] = o
                if c["ev"][i] is not None:
                    chunks.append(c["ev"][i])
                    o += len(c["ev"][i])
            offs_all.append(offs)
        inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()).cuda()
        if native_plan:  # every manager in one rsmi_fenc_plan_many call (host threads)
            ns_, _, sm_ = col.plan_many(encs, [c["lens"][cuts[ci][bi]:cuts[ci][bi + 1]]
                                               for ci, c in enumerate(cases)], offs_all, inbuf)
            S = FecEncoder.slot_stride_for(int(sm_.max()) - 128)
            nsl = int(ns_.sum())
        else:
            plans = [encs[ci].plan(c["lens"][cuts[ci][bi]:cuts[ci][bi + 1]], offs_all[ci], inbuf)
                     for ci, c in enumerate(cases)]
            # one stride for the shared array: every encoder's minimum, plus do_cook's tail
            S = FecEncoder.slot_stride_for(max(p.slot_stride_min for p in plans) - 128)
            nsl = sum(p.n_slots for p in plans)
        slots = torch.full((max(1, nsl) * S,), 0xEE, dtype=torch.uint8, device="cuda")
        out = torch.full_like(slots, 0x11) if cook else None
        ol = col.run_many(encs, slots, S, cook=ctx, seed=77 + bi, out=out)
        torch.cuda.synchronize()
        h = slots.cpu().numpy()
        hc = out.cpu().numpy() if cook else None
        olh = ol.cpu().numpy() if cook else None
        if cook:  # the collector draws IVs by the concatenated packet index
            from oracle.cpu import device_ivs
            ivs, ivls = device_ivs(77 + bi, 0, sum(len(e.packets_now()) for e in encs))
        q = 0
        for ci, c in enumerate(cases):
            pk = encs[ci].packets_now()
            a = cuts[ci][bi]
            for s, l, e in pk:
                plain = h[s * S + 120:s * S + 120 + l].tobytes()
                got[ci].append((plain, int(e) + a))
                if cook:
                    cl = int(olh[q])
                    assert cl > l
                    ck = hc[s * S + 120:s * S + 120 + cl].tobytes()
                    # byte for byte the oracle's do_cook with this packet's IV
                    # (a wrong or repeated IV index fails here, not in de_cook)
                    assert ck == cook_oracle.do_cook(plain, ivs[q, :ivls[q]].tobytes(), b"collector-key"), (ci, q)
                    st, back, nl = cook_oracle.de_cook(ck, b"collector-key")
                    assert st == 0 and back[:nl] == plain, (ci, q)
                q += 1
        del inbuf
    for ci, c in enumerate(cases):
        pk = [p for p, _ in got[ci]]
        assert [e for _, e in got[ci]] == list(c["pk_event"]), ci
        assert [len(p) for p in pk] == list(c["pk_len"]), ci
        assert hashlib.sha256(b"".join(pk)).digest() == c["sha"], ci
    col.close()
    for e in encs:
        e.close()


def _tiny_stream(seed, n):
    """Mode-0 events of 0-6 bytes (and timer flushes): a 20-shard group's
    blob then holds a few hundred records, so most shards overlap more than the
    fused framing cook's 8 records (kFuseRecs) and are left to k_frame."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 7, n).astype(np.int32)
    lens[rng.random(n) < 0.004] = -1
    pay = cook_payloads(seed, 0, n, np.maximum(lens, 0), 8)
    return lens, [None if lens[i] < 0 else pay[i, :lens[i]].tobytes() for i in range(n)]


def test_tiny_records_leave_shards_to_k_frame():
    """The planner's split for the fused run (no GPU): in a stream of tiny
    records, runs frame only a prefix of their data shards in list A
    (nfr < k) -- the case the GPU test below drives through k_frame."""
    from udpspeeder_amd.fec import FecEncoder
    lens, _ = _tiny_stream(77, 3000)
    enc = FecEncoder("20:10", 0, 1250, 200, seq0=9)
    p = enc.plan_host(lens, np.zeros(len(lens), np.uint64))
    runs = enc.packet_runs()
    g = p.groups
    k_of = {int(s0): int(k) for s0, k in zip(g["slot0"], g["k"])}
    short = [r for r in runs if int(r["nfr"]) < k_of[int(r["slot"])]]
    assert len(short) > len(runs) // 2
    assert all(int(r["ndata"]) <= int(r["nfr"]) for r in runs)
    enc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True])
def test_gpu_fused_cook_with_k_frame_leftovers(gpu, cook_oracle, packed):
    """A fused cooked run whose groups' shards overlap more than 8 records: the
    fused framing cook frames each group's leading shards, k_frame the rest,
    and every cooked packet equals the oracle's do_cook of the restatement's
    packet with the device-drawn IV, across batches cut mid-group."""
    import torch
    from oracle.cpu import device_ivs
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecEncoder
    lens, ev = _tiny_stream(77, 3000)
    n = len(lens)
    key = b"tiny key"
    enc = FecEncoder("20:10", 0, 1250, 200, seq0=9)
    em = EncodeManager("20:10", 0, 1250, 200, 9)
    exp = []
    for e in ev:
        em.input(e)
        exp += em.output()
    ctx = CookContext(key)
    got, ivs = [], []
    for bi, (a, b) in enumerate(zip([0, 1234], [1234, n])):
        offs = np.zeros(b - a, np.uint64)
        o, chunks = 0, []
        for i in range(a, b):
            offs[i - a] = o
            if ev[i] is not None:
                chunks.append(ev[i])
                o += len(ev[i])
        inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()).cuda()
        p = enc.plan(lens[a:b], offs, inbuf)
        S = p.slot_stride_min if packed else FecEncoder.slot_stride_for(p.slot_stride_min)
        slots = torch.full((max(1, p.n_slots) * S,), 0xEE, dtype=torch.uint8, device="cuda")
        if packed:
            po, ptot = enc.packed_offsets()
            out = torch.zeros(max(ptot, 16), dtype=torch.uint8, device="cuda")
            ol = enc.run_cooked_packed(slots, S, ctx, 50 + bi, out)
        else:
            out = torch.zeros(max(1, p.n_slots) * S, dtype=torch.uint8, device="cuda")
            ol = enc.run_cooked(slots, S, ctx, 50 + bi, out=out)
        torch.cuda.synchronize()
        ol = ol.cpu().numpy()[:len(p.packets)]
        h = out.cpu().numpy()
        iv, ivl = device_ivs(50 + bi, 0, len(p.packets))
        for i, (s, ln, _) in enumerate(p.packets):
            assert ol[i] == ln + 4 + ivl[i] + 1, (bi, i)
            o = int(po[i]) if packed else s * S + 120
            got.append(h[o:o + ol[i]].tobytes())
            ivs.append(iv[i, :ivl[i]].tobytes())
    assert len(got) == len(exp)
    bad = [i for i, (g_, e, v) in enumerate(zip(got, exp, ivs)) if g_ != cook_oracle.do_cook(e, v, key)]
    assert not bad, (len(bad), bad[:5])
    enc.close()


@pytest.mark.gpu
def test_gpu_collector_fused_with_k_frame_leftovers(gpu, cook_oracle):
    """The collector's fused cooked flush over managers whose groups leave
    shards to k_frame (over 8 records each): every manager's packets equal
    the restatement's, and every cooked packet de_cooks to them."""
    import torch
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecCollector, FecEncoder
    ncon, key = 8, b"tiny collector"
    streams = [_tiny_stream(100 + i, 700 + 50 * i) for i in range(ncon)]
    encs = [FecEncoder("20:10", 0, 1250, 200, seq0=3 + i) for i in range(ncon)]
    exp = []
    for i, (_, ev) in enumerate(streams):
        em = EncodeManager("20:10", 0, 1250, 200, 3 + i)
        pk = []
        for e in ev:
            em.input(e)
            pk += em.output()
        exp.append(pk)
    chunks, offs_all, o = [], [], 0
    for lens, ev in streams:
        offs = np.zeros(len(lens), np.uint64)
        for j, e in enumerate(ev):
            offs[j] = o
            if e is not None:
                chunks.append(e)
                o += len(e)
        offs_all.append(offs)
    inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()).cuda()
    plans = [encs[i].plan(streams[i][0], offs_all[i], inbuf) for i in range(ncon)]
    S = FecEncoder.slot_stride_for(max(p.slot_stride_min for p in plans))
    nsl = sum(p.n_slots for p in plans)
    slots = torch.full((max(1, nsl) * S,), 0xEE, dtype=torch.uint8, device="cuda")
    out = torch.full_like(slots, 0x11)
    col = FecCollector()
    ol = col.run_many(encs, slots, S, cook=CookContext(key), seed=5, out=out)
    torch.cuda.synchronize()
    h, hc, olh = slots.cpu().numpy(), out.cpu().numpy(), ol.cpu().numpy()
    from oracle.cpu import device_ivs
    ivs, ivls = device_ivs(5, 0, sum(len(e.packets_now()) for e in encs))
    q = 0
    for i in range(ncon):
        got = []
        for s, l, _ in encs[i].packets_now():
            plain = h[s * S + 120:s * S + 120 + l].tobytes()
            got.append(plain)
            ck = hc[s * S + 120:s * S + 120 + int(olh[q])].tobytes()
            assert ck == cook_oracle.do_cook(plain, ivs[q, :ivls[q]].tobytes(), key), (i, q)
            st, back, nl = cook_oracle.de_cook(ck, key)
            assert st == 0 and back[:nl] == plain, (i, q)
            q += 1
        assert got == exp[i], i
    col.close()
    for e in encs:
        e.close()


@pytest.mark.gpu
def test_gpu_collector_failure_after_remap_consumes_plans(gpu, monkeypatch):
    """rsmi_fenc_run_many rewrites the plans' slot references to the shared
    array before its uploads and launches; a failure after that point (here
    the rsmi_debug_fcol_fail hook) leaves no encoder planned, so a retry is a
    clean "encoder without a plan" error, not an out-of-bounds write.  After
    re-planning, the same encoders run and produce the reference's packets."""
    import torch
    from udpspeeder_amd._lib import RsmiError
    from udpspeeder_amd.fec import FecCollector, FecEncoder
    streams = [_tiny_stream(300 + i, 400) for i in range(3)]
    encs = [FecEncoder("20:10", 0, 1250, 200, seq0=11 + i) for i in range(3)]
    exp = []
    for i, (_, ev) in enumerate(streams):
        em = EncodeManager("20:10", 0, 1250, 200, 11 + i)
        pk = []
        for e in ev:
            em.input(e)
            pk += em.output()
        exp.append(pk)
    chunks, offs_all, o = [], [], 0
    for lens, ev in streams:
        offs = np.zeros(len(lens), np.uint64)
        for j, e in enumerate(ev):
            offs[j] = o
            if e is not None:
                chunks.append(e)
                o += len(e)
        offs_all.append(offs)
    inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()).cuda()
    col = FecCollector()

    def plan_all():
        ps = [encs[i].plan(streams[i][0], offs_all[i], inbuf) for i in range(3)]
        S = FecEncoder.slot_stride_for(max(p.slot_stride_min for p in ps))
        return S, torch.full((max(1, sum(p.n_slots for p in ps)) * S,), 0xEE, dtype=torch.uint8,
                             device="cuda")

    S, slots = plan_all()
    from udpspeeder_amd import lib
    lib().rsmi_debug_fcol_fail(1)
    try:
        with pytest.raises(RsmiError, match="injected"):
            col.run_many(encs, slots, S)
    finally:
        lib().rsmi_debug_fcol_fail(0)
    with pytest.raises(RsmiError, match="without a plan"):
        col.run_many(encs, slots, S)
    # the encoders' framing state is untouched by the failed runs: start the
    # streams again on fresh encoders of the same configuration
    for e in encs:
        e.close()
    encs[:] = [FecEncoder("20:10", 0, 1250, 200, seq0=11 + i) for i in range(3)]
    S, slots = plan_all()
    col.run_many(encs, slots, S)
    torch.cuda.synchronize()
    h = slots.cpu().numpy()
    for i in range(3):
        got = [h[s * S + 120:s * S + 120 + l].tobytes() for s, l, _ in encs[i].packets_now()]
        assert got == exp[i], i
    col.close()
    for e in encs:
        e.close()


def test_plan_many_equals_one_plan_each(fx):
    """rsmi_fenc_plan_many (every manager planned on a pool of host threads)
    makes exactly the decisions of one rsmi_fenc_plan per manager: the same
    input() returns, packet lists, groups and slot counts, over three batches
    of 60 managers' golden streams (plan-only encoders, no GPU)."""
    from udpspeeder_amd.fec import FecCollector, FecEncoder
    ncon = 60
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(ncon)]
    a = [FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"]) for c in cases]
    b = [FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"]) for c in cases]
    col = FecCollector()
    rng = np.random.default_rng(60)
    cuts = []
    for c in cases:
        n = len(c["lens"])
        x, y = sorted(rng.integers(1, n, 2))
        cuts.append([0, int(x), int(y), n])
    for bi in range(3):
        lens = [c["lens"][cuts[i][bi]:cuts[i][bi + 1]] for i, c in enumerate(cases)]
        offs = [np.zeros(len(l), np.uint64) for l in lens]
        ns, npk, sm = col.plan_many(a, lens, offs, None, nthreads=4)
        ret_all = col.last_ret
        q = 0
        for i in range(ncon):
            p = b[i].plan_host(lens[i], offs[i])
            assert (ns[i], npk[i], sm[i]) == (p.n_slots, len(p.packets), p.slot_stride_min), (bi, i)
            assert np.array_equal(ret_all[q:q + len(lens[i])], p.ret), (bi, i)
            q += len(lens[i])
            assert np.array_equal(a[i].packets_now(), p.packets), (bi, i)
            ga = a[i].groups_now() if hasattr(a[i], "groups_now") else None
            if ga is not None:
                for key in p.groups:
                    assert np.array_equal(ga[key], p.groups[key]), (bi, i, key)
    col.close()
    for e in a + b:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_gpu_collectors_split_over_device_list(fx, gpu, devices):
    """The send side sharded by connection (include/rsmi.h: one
    collector per device, each the managers of a contiguous connection range
    from rsmi_split_ranges balanced by bytes sent): 200 connections over the
    device list [0, 0] ([0, 0, 0]) -- one collector, slot array and host thread
    per entry, every thread on its device -- run concurrently per flush;
    every connection's packets equal the reference's."""
    import threading
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd.fec import FecCollector, FecEncoder
    ncon = 200
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(ncon)]
    encs = [FecEncoder(c["rs"], c["mode"], c["mtu"], c["ql"], seq0=c["seq0"]) for c in cases]
    ranges = u.rs.split_ranges(ncon, len(devices),
                               [int(np.maximum(c["lens"], 0).sum()) for c in cases])
    cols = [FecCollector() for _ in devices]
    rng = np.random.default_rng(201)
    cuts = []
    for c in cases:
        a, b = sorted(rng.integers(1, len(c["lens"]), 2))
        cuts.append([0, int(a), int(b), len(c["lens"])])
    got = [[] for _ in range(ncon)]
    errs = []

    def shard(r, bi):
        try:
            dev = devices[r]
            torch.cuda.set_device(dev)
            lo, hi = ranges[r]
            if hi <= lo:
                return
            chunks, offs_all, o = [], [], 0
            for ci in range(lo, hi):
                c = cases[ci]
                a, b = cuts[ci][bi], cuts[ci][bi + 1]
                offs = np.zeros(b - a, np.uint64)
                for i in range(a, b):
                    offs[i - a] = o
                    if c["ev"][i] is not None:
                        chunks.append(c["ev"][i])
                        o += len(c["ev"][i])
                offs_all.append(offs)
            inbuf = torch.from_numpy(np.frombuffer(b"".join(chunks) + bytes(32), np.uint8).copy()).cuda(dev)
            plans = [encs[ci].plan(cases[ci]["lens"][cuts[ci][bi]:cuts[ci][bi + 1]], offs_all[ci - lo], inbuf)
                     for ci in range(lo, hi)]
            S = FecEncoder.slot_stride_for(max(p.slot_stride_min for p in plans) - 128)
            nsl = sum(p.n_slots for p in plans)
            slots = torch.full((max(1, nsl) * S,), 0xEE, dtype=torch.uint8, device=f"cuda:{dev}")
            cols[r].run_many(encs[lo:hi], slots, S)
            torch.cuda.synchronize(dev)
            h = slots.cpu().numpy()
            for ci in range(lo, hi):
                a = cuts[ci][bi]
                for s, l, e in encs[ci].packets_now():
                    got[ci].append((h[s * S + 120:s * S + 120 + l].tobytes(), int(e) + a))
            del inbuf
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    for bi in range(3):
        ths = [threading.Thread(target=shard, args=(r, bi)) for r in range(len(devices))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert not errs, errs
    for ci, c in enumerate(cases):
        pk = [p for p, _ in got[ci]]
        assert [e for _, e in got[ci]] == list(c["pk_event"]), ci
        assert hashlib.sha256(b"".join(pk)).digest() == c["sha"], ci
    for col in cols:
        col.close()
    for e in encs:
        e.close()
