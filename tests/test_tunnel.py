"""GPU: the batched tunnel data path end to end over loopback UDP sockets
(udpspeeder_amd.tunnel, SURVEY §8f f4 with f1-f3): application datagrams ->
recvmmsg -> FEC framing + encode + cook on the GPU -> sendmmsg -> (packets
lost on the way) -> recvmmsg -> de_cook + FEC decode on the GPU -> sendmmsg
-> the application, which gets every datagram back, in order, byte for byte
(the reference's tunnel_client.cpp:41-80 and :110-160 per-packet loops)."""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sock(bind=True):
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 16 << 20)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 16 << 20)
    if bind:
        s.bind(("127.0.0.1", 0))
    return s


def _drop_in_groups(per_group):
    """Lose `per_group` packets of every FEC group (<= m: recoverable)."""
    def drop(p):
        slot = p.packets["slot"]
        lost = np.zeros(len(slot), bool)
        for s0, k, m in zip(p.groups["slot0"], p.groups["k"], p.groups["m"]):
            lose = min(per_group, int(m))
            # data shards first: the decoder must rebuild them
            lost |= (slot >= s0) & (slot < s0 + lose)
        return lost
    return drop


@pytest.mark.parametrize("mode,rs,loss", [(0, "20:10", 3), (1, "20:10", 2), (0, "1:3,2:4,10:6,20:10", 2)])
def test_tunnel_loopback_roundtrip(gpu, mode, rs, loss):
    from udpspeeder_amd import io
    from udpspeeder_amd.tunnel import Receiver, Sender
    rng = np.random.default_rng(mode * 7 + loss)
    app, c_in, c_out, s_in, s_out, sink = (_sock() for _ in range(6))
    n = 3000
    lens = rng.integers(0, 1201, n).astype(np.int32)
    lens[:3] = [0, 1, 1200]
    src = io.Slab(n, 1280)
    for i in range(n):
        src.slot(i, 0, int(lens[i]))[:] = rng.integers(0, 256, int(lens[i]), dtype=np.uint8)
        if lens[i] >= 4:
            src.slot(i, 0, 4)[:] = np.frombuffer(np.uint32(i).tobytes(), np.uint8)
    tx = Sender(rs, mode, 1250, 200, key=b"secret", batch=1024, max_len=1400)
    rx = Receiver(key=b"secret", batch=8192, max_len=1500)
    to_c, to_s, to_sink = (io.addr_of(*s.getsockname()) for s in (c_in, s_in, sink))
    drop = _drop_in_groups(loss)
    sent = 0
    for a in range(0, n, 500):  # the application writes in bursts
        io.send_batch(app, src, 0, lens[a:a + 500], slots=np.arange(a, min(n, a + 500)), to=to_c)
        while True:
            r, w = tx.step(c_in, c_out, to_s, timeout_ms=200, drop=drop)
            sent += w
            if r == 0:
                break
    sent += tx.flush(c_out, to_s, drop=drop)
    delivered = 0
    while True:
        r, w = rx.step(s_in, s_out, to_sink, timeout_ms=500)
        delivered += w
        if r == 0:
            break
    out = io.Slab(n + 8, 1536)
    got = io.recv_batch(sink, out, 0, 1500, n + 8, timeout_ms=2000)
    while len(got) < delivered:
        more = io.recv_batch(sink, _Tail(out, len(got)), 0, 1500, n + 8 - len(got), 2000)
        if len(more) == 0:
            break
        got = np.concatenate([got, more])
    assert delivered == n and len(got) == n
    want = [bytes(src.slot(i, 0, int(lens[i]))) for i in range(n)]
    have = [bytes(out.slot(i, 0, int(got[i]))) for i in range(n)]
    if mode == 0:
        assert have == want  # blobs come out whole, in order
    else:
        # mode 1 passes data packets through as they arrive and the rebuilt
        # ones after their group decodes (decode_fast_send, fec_manager.cpp:760-776)
        assert sorted(have) == sorted(want)


class _Tail:
    def __init__(self, slab, s):
        self.stride = slab.stride
        self.ptr = slab.ptr + s * slab.stride


# ---------------------------------------------------------------- interop
# The two halves of the tunnel against the REAL reference's halves
# (oracle/_ref: packet.cpp de_cook / do_cook, fec_manager.cpp's managers,
# compiled unmodified): our Sender's wire bytes must decode in the reference's
# receive path, and the reference's send path must decode in our Receiver --
# a framing or cook bug shared by both of our halves would pass the loopback
# test above but not these (tunnel_client.cpp:3-80 send side, :101-160
# receive side; packet.cpp:303-326).
def _ref_halves():
    from oracle.cpu import CookReference
    from oracle.fec_frame import FecReference
    if not (FecReference.available() and CookReference.available()):
        pytest.skip("reference build (oracle/_ref) absent")
    return FecReference(), CookReference()


def _datagrams(rng, n, mtu_payload=1200):
    lens = rng.integers(0, mtu_payload + 1, n)
    lens[:3] = [0, 1, mtu_payload]
    out = []
    for i, ln in enumerate(lens):
        b = bytearray(rng.integers(0, 256, int(ln), dtype=np.uint8).tobytes())
        if ln >= 4:
            b[:4] = np.uint32(i).tobytes()
        out.append(bytes(b))
    return out


def _drain(sock, max_len=1500):
    from udpspeeder_amd import io
    got = []
    while True:
        slab = io.Slab(4096, 1536)
        lens = io.recv_batch(sock, slab, 0, max_len, 4096, timeout_ms=300)
        if len(lens) == 0:
            return got
        got += [bytes(slab.slot(i, 0, int(lens[i]))) for i in range(len(lens))]


def _same(mode, have, want):
    if mode == 0:
        assert have == want  # blobs come out whole, in order
    else:
        assert sorted(have) == sorted(want)  # mode 1 fast-sends data packets


@pytest.mark.parametrize("mode,rs,loss", [(0, "20:10", 3), (1, "20:10", 2),
                                          (0, "1:3,2:4,10:6,20:10", 2)])
def test_sender_wire_decodes_in_reference(gpu, mode, rs, loss):
    """Our Sender (GPU framing + encode + cook) -> wire -> the reference's
    de_cook + fec_decode_manager_t: the application datagrams come out."""
    from udpspeeder_amd import io
    from udpspeeder_amd.tunnel import Sender
    fr, cr = _ref_halves()
    rng = np.random.default_rng(40 + mode * 3 + loss)
    data = _datagrams(rng, 2000)
    app, c_in, c_out, s_in = (_sock() for _ in range(4))
    src = io.Slab(len(data), 1280)
    for i, d in enumerate(data):
        src.slot(i, 0, len(d))[:] = np.frombuffer(d, np.uint8)
    lens = np.array([len(d) for d in data], np.int32)
    key = b"interop-key"
    tx = Sender(rs, mode, 1250, 200, key=key, batch=1024, max_len=1400)
    to_c, to_s = io.addr_of(*c_in.getsockname()), io.addr_of(*s_in.getsockname())
    drop = _drop_in_groups(loss)
    wire = []
    for a in range(0, len(data), 400):
        io.send_batch(app, src, 0, lens[a:a + 400], slots=np.arange(a, min(len(data), a + 400)),
                      to=to_c)
        while tx.step(c_in, c_out, to_s, timeout_ms=200, drop=drop)[0]:
            pass
        wire += _drain(s_in)
    tx.flush(c_out, to_s, drop=drop)
    wire += _drain(s_in)
    cr.config(key=key, flags=0)
    plain = []
    for pkt in wire:
        rc, buf, ln = cr.de_cook(pkt)
        assert rc == 0, "reference de_cook rejected a packet our GPU cooked"
        plain.append(buf[:ln])
    fr.config(rs, mode, 1250, 200)
    ret, outs, _ = fr.decode(plain)
    assert (ret == 0).all()
    _same(mode, outs, data)


@pytest.mark.parametrize("mode,rs,loss", [(0, "20:10", 3), (1, "20:10", 2),
                                          (0, "1:3,2:4,10:6,20:10", 2)])
def test_reference_wire_decodes_in_receiver(gpu, mode, rs, loss):
    """The reference's fec_encode_manager_t + do_cook -> wire (some packets of
    every group lost) -> our Receiver (GPU de_cook + gather + decode)."""
    from udpspeeder_amd import io
    from udpspeeder_amd.tunnel import Receiver
    fr, cr = _ref_halves()
    rng = np.random.default_rng(80 + mode * 3 + loss)
    data = _datagrams(rng, 2000)
    fr.config(rs, mode, 1250, 200)
    ret, pkts, _ = fr.encode(list(data) + [None])  # None: the FEC timer, input(0, 0)
    assert (ret[:-1] == 0).all()  # (the timer on an empty group returns -1, :226-229)
    # lose `loss` packets of every group, data shards first (header:
    # seq u32 | mode u8 | k u8 | m u8 | index u8, fec_manager.cpp:318-333)
    # (mode-1 data packets go out ahead with k = m = 0: their group's k, m
    # come from its parity packets, same seq)
    km = {}
    for p in pkts:
        if p[5]:
            km[bytes(p[:4])] = (p[5], p[6])
    keep = []
    for p in pkts:
        k, m = km.get(bytes(p[:4]), (0, 0))
        keep.append(not (k and p[7] < min(loss, m)))
    assert not all(keep)
    key = b"interop-key"
    cr.config(key=key, flags=0)
    cooked = [cr.do_cook(p) for p, kp in zip(pkts, keep) if kp]
    sender, s_in, s_out, sink = (_sock() for _ in range(4))
    src = io.Slab(len(cooked), 1536)
    for i, c in enumerate(cooked):
        src.slot(i, 0, len(c))[:] = np.frombuffer(c, np.uint8)
    clen = np.array([len(c) for c in cooked], np.int32)
    rx = Receiver(key=key, batch=8192, max_len=1500)
    to_s, to_sink = io.addr_of(*s_in.getsockname()), io.addr_of(*sink.getsockname())
    got = []
    for a in range(0, len(cooked), 1000):
        io.send_batch(sender, src, 0, clen[a:a + 1000], slots=np.arange(a, min(len(cooked), a + 1000)),
                      to=to_s)
        while rx.step(s_in, s_out, to_sink, timeout_ms=200)[0]:
            pass
        got += _drain(sink)
    _same(mode, got, data)
