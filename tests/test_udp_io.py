"""CPU: batched UDP I/O (include/rsmi_io.h) over loopback
sockets -- the recvmmsg / sendmmsg replacement of the reference's per-datagram
recvfrom / recv (tunnel_client.cpp:47,119) and sendto (packet.cpp:149-231):
every byte and length arrives, in order, with the sender's address; a datagram
longer than max_len is flagged -1 as the callbacks drop it
(tunnel_client.cpp:50-53); a timeout returns 0; batches larger than one
recvmmsg / sendmmsg call (1024 messages) work."""
import socket

import numpy as np
import pytest

from udpspeeder_amd import io


def _pair():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.bind(("127.0.0.1", 0))
    return rx, tx


def test_roundtrip_lengths_bytes_order_and_sender():
    rx, tx = _pair()
    rng = np.random.default_rng(1)
    n, S, off, mx = 700, 1536, 120, 1400
    lens = rng.integers(0, mx + 1, n).astype(np.int32)
    lens[:4] = [0, 1, mx, 15]
    src = io.Slab(n, S)
    for i in range(n):
        src.slot(i, off, int(lens[i]))[:] = rng.integers(0, 256, int(lens[i]), dtype=np.uint8)
    to = io.addr_of(*rx.getsockname())
    assert io.send_batch(tx, src, off, lens, to=to) == n
    dst = io.Slab(n, S)
    got, addrs = io.recv_batch(rx, dst, off, mx, n, timeout_ms=2000, with_addr=True)
    while len(got) < n:  # a later call takes the rest
        more, a2 = io.recv_batch(rx, _tail(dst, len(got)), off, mx, n - len(got), 2000, True)
        got = np.concatenate([got, more])
        addrs += a2
    assert (got == lens).all()
    for i in range(n):
        assert (dst.slot(i, off, int(lens[i])) == src.slot(i, off, int(lens[i]))).all()
    assert all(io.addr_to_tuple(a) == tx.getsockname() for a in addrs)


class _tail:
    """A view of a slab from slot s on (for a second receive call)."""

    def __init__(self, slab, s):
        self.stride = slab.stride
        self.ptr = slab.ptr + s * slab.stride


def test_oversize_flagged_and_timeout():
    rx, tx = _pair()
    tx.sendto(b"x" * 300, rx.getsockname())
    tx.sendto(b"y" * 100, rx.getsockname())
    slab = io.Slab(4, 512)
    got = io.recv_batch(rx, slab, 0, 200, 4, timeout_ms=2000)
    assert list(got) == [-1, 100]  # > max_len: dropped like data_len == max_data_len + 1
    assert bytes(slab.slot(1, 0, 100)) == b"y" * 100
    assert len(io.recv_batch(rx, slab, 0, 200, 4, timeout_ms=50)) == 0


def test_skips_negative_lengths_and_uses_slot_list():
    rx, tx = _pair()
    src = io.Slab(8, 64)
    for i in range(8):
        src.slot(i)[:] = i
    n = io.send_batch(tx, src, 0, [10, -1, 20, 5], slots=[7, 0, 3, 1], to=io.addr_of(*rx.getsockname()))
    assert n == 3
    dst = io.Slab(4, 64)
    got = io.recv_batch(rx, dst, 0, 32, 4, timeout_ms=2000)
    assert list(got) == [10, 20, 5]
    assert (dst.slot(0, 0, 10) == 7).all() and (dst.slot(1, 0, 20) == 3).all() and (dst.slot(2, 0, 5) == 1).all()


def test_more_than_one_call_chunk():
    rx, tx = _pair()
    n, S = 3000, 128
    src = io.Slab(n, S)
    lens = np.full(n, 64, np.int32)
    for i in range(n):
        src.slot(i, 0, 4)[:] = np.frombuffer(np.uint32(i).tobytes(), np.uint8)
    assert io.send_batch(tx, src, 0, lens, to=io.addr_of(*rx.getsockname())) == n
    dst = io.Slab(n, S)
    got = io.recv_batch(rx, dst, 0, 100, n, timeout_ms=2000)
    assert len(got) == n and (got == 64).all()
    ids = [int(np.frombuffer(bytes(dst.slot(i, 0, 4)), np.uint32)[0]) for i in range(n)]
    assert ids == list(range(n))


def test_send_from_pointers():
    rx, tx = _pair()
    bufs = [np.frombuffer(bytes([i]) * (10 + i), np.uint8).copy() for i in range(5)]
    ptrs = [b.ctypes.data for b in bufs]
    assert io.send_ptrs(tx, ptrs, [len(b) for b in bufs[:4]] + [-1], io.addr_of(*rx.getsockname())) == 4
    dst = io.Slab(8, 64)
    got = io.recv_batch(rx, dst, 0, 32, 8, timeout_ms=2000)
    assert list(got) == [10, 11, 12, 13]
    for i in range(4):
        assert bytes(dst.slot(i, 0, 10 + i)) == bytes([i]) * (10 + i)


def test_bad_args():
    from udpspeeder_amd._lib import RsmiError
    rx, _ = _pair()
    slab = io.Slab(2, 64)
    with pytest.raises(RsmiError):
        io.recv_batch(rx, slab, 0, 64, 2, timeout_ms=0)  # slot needs max_len + 1 bytes


def test_one_bad_datagram_does_not_stop_the_batch():
    """A datagram the kernel rejects on its own (EMSGSIZE here; ECONNREFUSED
    after an ICMP port-unreachable is the same case) is dropped and the rest of
    the batch still goes out, as the reference's per-packet sendto does
    (packet.cpp:149-162); only a batch of which nothing went out is an error."""
    from udpspeeder_amd._lib import RsmiError
    rx, tx = _pair()
    S = 70000
    src = io.Slab(4, S)
    for i in range(4):
        src.slot(i)[:] = i + 1
    to = io.addr_of(*rx.getsockname())
    assert io.send_batch(tx, src, 0, [10, 66000, 20, 30], to=to) == 3
    dst = io.Slab(4, 64)
    got = io.recv_batch(rx, dst, 0, 32, 4, timeout_ms=2000)
    assert list(got) == [10, 20, 30]
    assert (dst.slot(1, 0, 20) == 3).all() and (dst.slot(2, 0, 30) == 4).all()
    with pytest.raises(RsmiError):
        io.send_batch(tx, src, 0, [66000, 66000], to=to)


def test_connection_refused_mid_batch():
    """Connected socket, peer port closed: the ICMP error surfaces on a later
    send as ECONNREFUSED for one datagram; the call still returns a count."""
    rx, tx = _pair()
    port = rx.getsockname()[1]
    rx.close()
    tx.connect(("127.0.0.1", port))
    src = io.Slab(64, 64)
    total = 0
    for _ in range(4):
        n = io.send_batch(tx, src, 0, np.full(64, 16, np.int32))
        assert 0 < n <= 64
        total += n
    assert total < 4 * 64  # at least one refused datagram was skipped, not fatal


def test_socket_error_stops_the_batch():
    """A failure of the socket itself (here EDESTADDRREQ: an unconnected socket
    and no destination) is not a per-datagram drop: every later datagram would
    fail the same way, so the call reports an I/O error at once instead of
    spending one syscall per datagram."""
    import socket
    import time
    from udpspeeder_amd._lib import RsmiError
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        src = io.Slab(4096, 64)
        t0 = time.perf_counter()
        with pytest.raises(RsmiError, match="sendmmsg"):
            io.send_batch(tx, src, 0, np.full(4096, 16, np.int32))
        assert time.perf_counter() - t0 < 0.5
    finally:
        tx.close()


def test_wrong_family_destination_is_per_datagram():
    """EINVAL / EAFNOSUPPORT (an IPv6 destination on an IPv4 socket) is a
    failure of that datagram's address, not of the socket: each datagram is
    tried and dropped (packet.cpp:143-162 logs and carries on); with none sent
    the call reports an I/O error naming sendmmsg."""
    import socket
    from udpspeeder_amd._lib import RsmiError
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        src = io.Slab(8, 64)
        import ctypes as C
        import struct
        to6 = io.rsmi_udp_addr()
        raw = (struct.pack("=H", socket.AF_INET6) + struct.pack("!H", 9) + bytes(4)
               + socket.inet_pton(socket.AF_INET6, "::1") + bytes(4))
        C.memmove(to6.storage, raw, len(raw))
        to6.len = len(raw)
        with pytest.raises(RsmiError, match="sendmmsg"):
            io.send_batch(tx, src, 0, np.full(8, 16, np.int32), to=to6)
    finally:
        tx.close()
