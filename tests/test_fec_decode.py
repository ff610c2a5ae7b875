"""Receive side of the FEC framing: fec_decode_manager_t.

CPU tests pin the Python restatement (oracle/fec_frame.py:DecodeManager) to the
REAL reference decoder -- through the committed fixtures
(tests/golden/fec_decode.npz, oracle/gen_golden_fec.py) and, where the
reference build is present, live on long runs whose delays exceed the
2000-buffer ring -- and check librsmi.so's host planner (return codes) without
a GPU.  GPU tests run the batched decoder (plan -> gather/decode/pack on the
GPU -> outputs) and compare every output packet with the fixtures and the
restatement, with batches cut at arbitrary packets so groups straddle batches.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle.fec_frame import DecodeManager, EncodeManager, FecReference, lossy_channel
from oracle.gen_golden_fec import DEC_CASES, dec_channel

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fec_decode.npz")
NAMES = [c[0] for c in DEC_CASES]


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(GOLDEN))


def _case(fx, name):
    chan = dec_channel(name)
    h = hashlib.sha256(b"".join(len(p).to_bytes(4, "little") + p for p in chan)).digest()
    assert h == fx[f"{name}__chan_sha256"].tobytes(), "channel regeneration drifted"
    full = fx.get(f"{name}__out_bytes")
    exp = None
    if full is not None:
        off = np.concatenate([[0], np.cumsum(fx[f"{name}__out_len"])])
        b = full.tobytes()
        exp = [b[off[i]:off[i + 1]] for i in range(len(off) - 1)]
    return dict(chan=chan, ret=list(fx[f"{name}__ret"]), out_len=list(fx[f"{name}__out_len"]),
                out_event=list(fx[f"{name}__out_event"]), sha=fx[f"{name}__sha256"].tobytes(),
                exp=exp)


def _oracle_run(chan, now=None):
    dm = DecodeManager()
    ret, out, ev = [], [], []
    for i, p in enumerate(chan):
        if now is not None:
            dm.now = now[i]
        ret.append(dm.input(p))
        o = dm.output()
        out += o
        ev += [i] * len(o)
    return ret, out, ev


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_fixtures(fx, name):
    c = _case(fx, name)
    ret, out, ev = _oracle_run(c["chan"])
    assert ret == c["ret"]
    assert ev == c["out_event"]
    assert [len(p) for p in out] == c["out_len"]
    assert hashlib.sha256(b"".join(out)).digest() == c["sha"]
    if c["exp"] is not None:
        assert out == c["exp"]


def _pack(chan):
    lens = np.array([len(p) for p in chan], np.int32)
    offs = np.zeros(len(chan), np.uint64)
    o = 0
    for i, p in enumerate(chan):
        offs[i] = o
        o += (len(p) + 15) // 16 * 16 + 16
    host = np.zeros(o + 64, np.uint8)
    for i, p in enumerate(chan):
        host[offs[i]:offs[i] + len(p)] = np.frombuffer(p, np.uint8)
    return host, lens, offs


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("nbatch", [1, 3])
def test_planner_ret_matches_reference(fx, name, nbatch):
    """librsmi.so's planner without a GPU: every input() return value."""
    from udpspeeder_amd.fec import FecDecoder
    c = _case(fx, name)
    host, lens, offs = _pack(c["chan"])
    dec = FecDecoder()
    cuts = np.linspace(0, len(lens), nbatch + 1).astype(int)
    ret = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        ret += list(dec.plan(host, lens[a:b], offs[a:b]).ret)
    assert ret == c["ret"]
    dec.close()


@pytest.mark.parametrize("nthreads", [1, 4])
def test_planner_plan_many_matches_reference(fx, nthreads):
    """rsmi_fdec_plan_many (every decoder planned on a pool of host threads):
    each decoder's return codes over 3 batches equal the reference's."""
    from udpspeeder_amd.fec import FecDecodeCollector, FecDecoder
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(2 * len(NAMES))]
    packed = [_pack(c["chan"]) for c in cases]
    decs = [FecDecoder() for _ in cases]
    col = FecDecodeCollector()
    ret = [[] for _ in cases]
    for bi in range(3):
        cuts = [np.linspace(0, len(p[1]), 4).astype(int)[bi:bi + 2] for p in packed]
        plans = col.plan_many(decs, [p[0] for p in packed], [p[1][a:b] for p, (a, b) in zip(packed, cuts)],
                              [p[2][a:b] for p, (a, b) in zip(packed, cuts)], nthreads=nthreads)
        for i, pl in enumerate(plans):
            ret[i] += list(pl.ret)
    for i, c in enumerate(cases):
        assert ret[i] == c["ret"], i
    col.close()
    for d in decs:
        d.close()


def _long_run(mode, rs, seed, n=6000, lmax=900):
    rng = np.random.default_rng(seed)
    em = EncodeManager(rs, mode, 1250, 200, seed)
    pk = []
    for i in range(n):
        if rng.random() < 0.02:
            em.input(None)
        else:
            em.input(rng.integers(0, 256, int(rng.integers(0, lmax + 1)), dtype=np.uint8).tobytes())
        pk += em.output()
    return lossy_channel(pk, seed, loss=0.2, dup=0.05, swap=0.1, delay=0.01, delay_by=2100,
                         replay=0.01, trunc=0.01, garbage=0.01)


@pytest.mark.skipif(not FecReference.available(), reason="reference build absent")
@pytest.mark.parametrize("mode,rs", [(0, "20:10"), (1, "1:3,2:4,10:6,20:10")])
def test_oracle_matches_live_reference_with_ring_evictions(mode, rs):
    chan = _long_run(mode, rs, 31 + mode)
    fr = FecReference()
    r_ret, r_out, r_ev = fr.decode(chan)
    ret, out, ev = _oracle_run(chan)
    assert ret == list(r_ret) and ev == list(r_ev) and out == r_out


@pytest.mark.parametrize("mode,rs,seed", [(0, "20:10", 41), (1, "1:3,2:4,10:6,20:10", 42), (0, "1:3,2:4,10:6,20:10", 43)])
def test_planner_long_runs_with_evictions_match_oracle(mode, rs, seed):
    """librsmi.so's planner without a GPU on 6,000-event runs with loss,
    duplicates, swaps, delays past the 2,000-slot ring (evictions), replays,
    truncations and garbage, cut into uneven batches: every input() return
    value equals the restatement's (pinned to the live reference above).
    Exercises the planner's flat maps and its memoised lookups and evictions
    (fec_dec.cpp SeqMap / SeqMemo / EvictMemo) where groups interleave."""
    from udpspeeder_amd.fec import FecDecoder
    chan = _long_run(mode, rs, seed)
    ret, _, _ = _oracle_run(chan)
    host, lens, offs = _pack(chan)
    dec = FecDecoder()
    cuts = [0, 1, 700, 701, 2900, 4321, len(chan)]
    got = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        got += list(dec.plan(host, lens[a:b], offs[a:b]).ret)
    assert got == ret
    dec.close()


def test_planner_anti_replay_timeout_matches_oracle():
    """anti_replay_timeout (120 s): replays older than it are accepted again."""
    from udpspeeder_amd.fec import FecDecoder
    chan = _long_run(1, "20:10", 5, n=1500)
    chan = chan + chan[:400]  # replayed, some after the window
    now = np.zeros(len(chan), np.int64)
    now[len(chan) - 400:] = np.linspace(60_000, 300_000, 400).astype(np.int64)
    ret, _, _ = _oracle_run(chan, now)
    host, lens, offs = _pack(chan)
    dec = FecDecoder()
    got = []
    # one packet per plan where the clock moves, as the reference reads it per input()
    got += list(dec.plan(host, lens[:len(chan) - 400], offs[:len(chan) - 400], now_ms=0).ret)
    for i in range(len(chan) - 400, len(chan)):
        got += list(dec.plan(host, lens[i:i + 1], offs[i:i + 1], now_ms=int(now[i])).ret)
    assert got == ret
    dec.close()


def _gpu_run(chan, cuts, torch):
    from udpspeeder_amd.fec import FecDecoder
    host, lens, offs = _pack(chan)
    dev = torch.from_numpy(host).cuda()
    dec = FecDecoder()
    ret, out = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        p = dec.plan(host, lens[a:b], offs[a:b], dev)
        ret += list(p.ret)
        dec.run()
        out += [(bts, e + a) for bts, e in dec.outputs()]
    dec.close()
    return ret, out


def _gpu_run_pipelined(chan, cuts, torch):
    """plan(i+1) and run(i+1) before batch i's outputs are taken, batches on
    two alternating streams (the decoder's double-buffered batches)."""
    from udpspeeder_amd.fec import FecDecoder
    host, lens, offs = _pack(chan)
    dev = torch.from_numpy(host).cuda()
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dec = FecDecoder()
    ret, out = [], []
    starts = []
    for bi, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        p = dec.plan(host, lens[a:b], offs[a:b], dev)
        ret += list(p.ret)
        dec.run(stream=streams[bi % 2])
        starts.append(a)
        if bi:  # the previous batch's outputs, after this batch was planned and launched
            out += [(bts, e + starts[bi - 1]) for bts, e in dec.outputs()]
    out += [(bts, e + starts[-1]) for bts, e in dec.outputs()]
    dec.close()
    return ret, out


def _cuts(n, nbatch, seed):
    rng = np.random.default_rng(seed)
    if nbatch == 1:
        return np.array([0, n])
    return np.unique(np.concatenate([[0, n], rng.integers(0, n, nbatch - 1)]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("nbatch", [1, 4])
def test_gpu_decoder_matches_reference(fx, gpu, name, nbatch):
    import torch
    c = _case(fx, name)
    ret, out = _gpu_run(c["chan"], _cuts(len(c["chan"]), nbatch, len(name)), torch)
    assert ret == c["ret"]
    assert [e for _, e in out] == c["out_event"]
    assert [len(b) for b, _ in out] == c["out_len"]
    if c["exp"] is not None:
        bad = [i for i, ((b, _), x) in enumerate(zip(out, c["exp"])) if b != x]
        assert not bad, (len(bad), bad[:5])
    assert hashlib.sha256(b"".join(b for b, _ in out)).digest() == c["sha"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,rs", [(0, "20:10"), (0, "1:3,2:4,10:6,20:10"), (1, "20:10"),
                                     (1, "1:3,2:4,10:6,20:10")])
def test_gpu_decoder_matches_oracle_long(gpu, mode, rs):
    import torch
    chan = _long_run(mode, rs, 77 + mode)
    ret, out, ev = _oracle_run(chan)
    g_ret, g_out = _gpu_run(chan, _cuts(len(chan), 5, 3), torch)
    assert g_ret == ret
    assert [e for _, e in g_out] == ev
    bad = [i for i, ((b, _), x) in enumerate(zip(g_out, out)) if b != x]
    assert not bad, (len(bad), bad[:5])


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 7])
@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_decoder_threaded_outputs(gpu, monkeypatch, mode, threads):
    """Output resolution split over 7 threads (every batch, however small) keeps
    the reference's output order and bytes."""
    import torch
    monkeypatch.setenv("RSMI_FDEC_PAR_MIN", "1")
    monkeypatch.setenv("RSMI_HOST_THREADS", str(threads))
    chan = _long_run(mode, "1:3,2:4,10:6,20:10", 91 + mode)
    ret, out, ev = _oracle_run(chan)
    g_ret, g_out = _gpu_run(chan, _cuts(len(chan), 5, 4), torch)
    assert g_ret == ret
    assert [e for _, e in g_out] == ev
    assert [b for b, _ in g_out] == out


@pytest.mark.gpu
@pytest.mark.parametrize("mode,rs", [(0, "20:10"), (1, "1:3,2:4,10:6,20:10")])
def test_gpu_decoder_pipelined_two_streams(gpu, mode, rs):
    import torch
    chan = _long_run(mode, rs, 55 + mode)
    ret, out, ev = _oracle_run(chan)
    g_ret, g_out = _gpu_run_pipelined(chan, _cuts(len(chan), 6, 8), torch)
    assert g_ret == ret
    assert [e for _, e in g_out] == ev
    bad = [i for i, ((b, _), x) in enumerate(zip(g_out, out)) if b != x]
    assert not bad, (len(bad), bad[:5])


@pytest.mark.gpu
def test_gpu_per_call_interface(gpu):
    """input()/output() one packet at a time (misc.cpp:409-425's loop)."""
    from udpspeeder_amd.fec import FecDecoder
    chan = _long_run(0, "3:2", 9, n=300, lmax=50)
    dm = DecodeManager()
    dec = FecDecoder()
    for p in chan:
        assert dec.input(p) == dm.input(p)
        assert dec.output() == dm.output()
    dec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("native_plan", [False, True])
def test_gpu_decode_collector_200_connections_match_reference(fx, gpu, native_plan):
    """The receive-side collector (rsmi_fdec_run_many): 200 decoders, one per
    connection (connection.h:244-245, max_conn_num = 200, common.h:112), each
    fed its own golden channel (case i % len(DEC_CASES), cut into 3 batches at its own
    points, so groups straddle batches through each decoder's ring), planned
    one by one, run together: every connection's return codes, output events
    and output bytes equal the reference's."""
    import torch
    from udpspeeder_amd.fec import FecDecodeCollector, FecDecoder
    ncon = 200
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(ncon)]
    packed = [_pack(c["chan"]) for c in cases]
    devs = [torch.from_numpy(h).cuda() for h, _, _ in packed]
    decs = [FecDecoder() for _ in range(ncon)]
    col = FecDecodeCollector()
    rng = np.random.default_rng(9)
    cuts = []
    for c in cases:
        n = len(c["chan"])
        a, b = sorted(rng.integers(1, n, 2))
        cuts.append([0, int(a), int(b), n])
    ret = [[] for _ in range(ncon)]
    out = [[] for _ in range(ncon)]
    for bi in range(3):
        if native_plan:  # rsmi_fdec_plan_many: all 200 planned on host threads
            sl = [slice(cuts[ci][bi], cuts[ci][bi + 1]) for ci in range(ncon)]
            plans = col.plan_many(decs, [p[0] for p in packed], [p[1][s] for p, s in zip(packed, sl)],
                                  [p[2][s] for p, s in zip(packed, sl)], devs)
            for ci in range(ncon):
                ret[ci] += list(plans[ci].ret)
        else:
            for ci in range(ncon):
                host, lens, offs = packed[ci]
                a, b = cuts[ci][bi], cuts[ci][bi + 1]
                ret[ci] += list(decs[ci].plan(host, lens[a:b], offs[a:b], devs[ci]).ret)
        col.run_many(decs)
        for ci in range(ncon):
            a = cuts[ci][bi]
            out[ci] += [(bts, e + a) for bts, e in decs[ci].outputs()]
    for ci, c in enumerate(cases):
        assert ret[ci] == c["ret"], ci
        assert [e for _, e in out[ci]] == c["out_event"], ci
        assert [len(b) for b, _ in out[ci]] == c["out_len"], ci
        assert hashlib.sha256(b"".join(b for b, _ in out[ci])).digest() == c["sha"], ci
    col.close()
    for d in decs:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_gpu_decode_collectors_split_over_device_list(fx, gpu, devices):
    """The receive side sharded by connection (include/rsmi.h: one
    collector per device, each the decoders of a contiguous connection range
    from rsmi_split_ranges balanced by bytes received): 200 connections over
    the device list [0, 0] ([0, 0, 0]) -- one collector and one host thread per
    entry, every thread on its device -- run concurrently per flush; every
    connection's return codes, output events and bytes equal the reference's."""
    import threading
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd.fec import FecDecodeCollector, FecDecoder
    ncon = 200
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(ncon)]
    packed = [_pack(c["chan"]) for c in cases]
    devs_t = [torch.from_numpy(h).cuda(devices[0]) for h, _, _ in packed]
    ranges = u.rs.split_ranges(ncon, len(devices), [int(p[1].sum()) for p in packed])
    decs = [FecDecoder() for _ in range(ncon)]
    cols = [FecDecodeCollector() for _ in devices]
    rng = np.random.default_rng(19)
    cuts = []
    for c in cases:
        a, b = sorted(rng.integers(1, len(c["chan"]), 2))
        cuts.append([0, int(a), int(b), len(c["chan"])])
    ret = [[] for _ in range(ncon)]
    out = [[] for _ in range(ncon)]
    errs = []

    def shard(r, bi):
        try:
            torch.cuda.set_device(devices[r])
            lo, hi = ranges[r]
            for ci in range(lo, hi):
                host, lens, offs = packed[ci]
                a, b = cuts[ci][bi], cuts[ci][bi + 1]
                ret[ci] += list(decs[ci].plan(host, lens[a:b], offs[a:b], devs_t[ci]).ret)
            if hi > lo:
                cols[r].run_many(decs[lo:hi])
            for ci in range(lo, hi):
                a = cuts[ci][bi]
                out[ci] += [(bts, e + a) for bts, e in decs[ci].outputs()]
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
        assert ret[ci] == c["ret"], ci
        assert [e for _, e in out[ci]] == c["out_event"], ci
        assert hashlib.sha256(b"".join(b for b, _ in out[ci])).digest() == c["sha"], ci
    for col in cols:
        col.close()
    for d in decs:
        d.close()


@pytest.mark.gpu
def test_gpu_decode_collector_reused_set_is_detected(fx, gpu):
    """A decoder run by collector call t and left out of calls t+1 and t+2:
    call t+2 reuses the set that held its rows, so its outputs are refused
    with an error (they pointed at overwritten or freed memory);
    read before that, they are the reference's."""
    import torch
    from udpspeeder_amd._lib import RsmiError
    from udpspeeder_amd.fec import FecDecodeCollector, FecDecoder
    cases = [_case(fx, NAMES[i % len(NAMES)]) for i in range(3)]
    packed = [_pack(c["chan"]) for c in cases]
    devs = [torch.from_numpy(h).cuda() for h, _, _ in packed]
    decs = [FecDecoder() for _ in range(3)]
    col = FecDecodeCollector()

    def plan(i):
        host, lens, offs = packed[i]
        return list(decs[i].plan(host, lens, offs, devs[i]).ret)

    assert plan(0) == cases[0]["ret"]
    col.run_many([decs[0]])            # call t: decoder 0's rows in set A
    plan(1)
    col.run_many([decs[1]])            # call t+1: set B
    first = decs[1].outputs()          # (read in time: fine)
    assert hashlib.sha256(b"".join(b for b, _ in first)).digest() == cases[1]["sha"]
    plan(2)
    col.run_many([decs[2]])            # call t+2: set A again
    with pytest.raises(RsmiError, match="reused"):
        decs[0].outputs()
    assert hashlib.sha256(b"".join(b for b, _ in decs[2].outputs())).digest() == cases[2]["sha"]
    col.close()
    for d in decs:
        d.close()
