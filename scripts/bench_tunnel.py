"""End to end over loopback UDP (SURVEY §8f f4 with f1-f3): the batched tunnel
data path of udpspeeder_amd.tunnel, one GPU.

    app --UDP--> Sender (recvmmsg, FEC framing + encode + cook on the GPU,
    sendmmsg) --UDP--> Receiver (recvmmsg, de_cook + FEC decode on the GPU,
    sendmmsg) --UDP--> sink

Four threads, one per stage, with a credit window so the loopback socket
buffers never overflow (UDP would drop): the application sends burst i+2 only
once the sink has all of burst i.  Workload: mode 0, -f 20:10, mtu 1250,
1200-byte datagrams, a key (every transform on); `--loss` drops that many
packets of every FEC group between the two ends (the decoder rebuilds them).
Reports datagrams/s delivered end to end and each stage's busy time.

    python scripts/bench_tunnel.py [--packets 262144] [--burst 8192] [--loss 0]
"""
import argparse
import json
import os
import socket
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sock(buf):
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, buf)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, buf)
    s.bind(("127.0.0.1", 0))
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=262144)
    ap.add_argument("--burst", type=int, default=8192)
    ap.add_argument("--len", type=int, default=1200)
    ap.add_argument("--loss", type=int, default=0, help="packets lost per FEC group")
    args = ap.parse_args()
    import torch
    from udpspeeder_amd import io
    from udpspeeder_amd.tunnel import Receiver, Sender
    try:
        rmem = int(open("/proc/sys/net/core/rmem_max").read())
    except OSError:
        rmem = 212992
    buf = max(rmem, 1 << 20)
    # two bursts in flight must fit the smallest socket buffer (cooked packets
    # are ~1.55x the datagrams with parity and cook tails)
    burst = max(256, min(args.burst, buf // (2 * 2 * (args.len + 120))))
    n = args.packets // burst * burst
    app, c_in, c_out, s_in, s_out, sink = (_sock(buf) for _ in range(6))
    to_c, to_s, to_sink = (io.addr_of(*s.getsockname()) for s in (c_in, s_in, sink))
    src = io.Slab(burst, 1280)
    rng = np.random.default_rng(1)
    for i in range(burst):
        src.slot(i, 0, args.len)[:] = rng.integers(0, 256, args.len, dtype=np.uint8)
    tx = Sender("20:10", 0, 1250, 200, key=b"bench-key", batch=burst, max_len=1400)
    rx = Receiver(key=b"bench-key", batch=4 * burst, max_len=1500)
    drop = None
    if args.loss:
        def drop(p):
            slot = p.packets["slot"]
            lost = np.zeros(len(slot), bool)
            for s0 in p.groups["slot0"]:
                lost |= (slot >= s0) & (slot < s0 + args.loss)
            return lost
    got = [0]
    busy = {"sender": 0.0, "receiver": 0.0}
    cv = threading.Condition()
    done = threading.Event()
    lens = np.full(burst, args.len, np.int32)

    def app_thread():
        for b in range(n // burst):
            with cv:
                cv.wait_for(lambda: got[0] >= (b - 1) * burst)
            io.send_batch(app, src, 0, lens, to=to_c)

    def sender_thread():
        torch.cuda.set_device(0)
        while not done.is_set():
            t = time.perf_counter()
            r, _ = tx.step(c_in, c_out, to_s, timeout_ms=8, drop=drop)
            if r:
                busy["sender"] += time.perf_counter() - t
            else:  # the FEC timer (fec_par.timeout, 8 ms): close the open group
                tx.flush(c_out, to_s, drop=drop)

    def receiver_thread():
        torch.cuda.set_device(0)
        while not done.is_set():
            t = time.perf_counter()
            r, _ = rx.step(s_in, s_out, to_sink, timeout_ms=20)
            if r:
                busy["receiver"] += time.perf_counter() - t

    class View:
        stride = 1536
        def __init__(self, t):
            self.ptr = t.data_ptr()
    sink_buf = torch.empty(4 * burst * 1536, dtype=torch.uint8).pin_memory()
    sv = View(sink_buf)

    def sink_thread():
        while got[0] < n:
            m = len(io.recv_batch(sink, sv, 0, 1500, 4 * burst, timeout_ms=5000))
            if m == 0:
                break
            with cv:
                got[0] += m
                cv.notify_all()

    th = [threading.Thread(target=f) for f in (sender_thread, receiver_thread, sink_thread)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    a = threading.Thread(target=app_thread)
    a.start()
    th[2].join()
    t1 = time.perf_counter()
    done.set()
    a.join()
    for t in th[:2]:
        t.join()
    wall = t1 - t0
    print(json.dumps({
        "workload": f"loopback UDP, mode 0 -f 20:10 mtu 1250, {args.len}-B datagrams, key on, "
                    f"{args.loss} packets lost per group, bursts of {burst}",
        "datagrams": n, "delivered": got[0], "wall_s": round(wall, 3),
        "datagrams_per_s": round(got[0] / wall, 1),
        "payload_Gbit_per_s": round(got[0] * args.len * 8 / wall / 1e9, 2),
        "sender_busy_s": round(busy["sender"], 3), "receiver_busy_s": round(busy["receiver"], 3),
        "socket_buffer_bytes": buf}))
    return 0 if got[0] == n else 1


if __name__ == "__main__":
    sys.exit(main())
