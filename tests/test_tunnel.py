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
