"""Several GPUs behind the host-memory entry points (SURVEY.md §8e,
include/rsmi.h rsmi_use_devices): the range split on the CPU, and on the GPU
the split pipelines bit-exact against the single-device path and the oracle.
On the 1-GPU box the device list [0, 0] (and [0, 0, 0]) runs two (three)
workers with their own streams and buffers on one device: the same partition,
threads and joins as eight devices."""
import numpy as np
import pytest

import udpspeeder_amd as u
from udpspeeder_amd import shard


@pytest.mark.parametrize("n,parts", [(0, 1), (1, 3), (7, 2), (65536, 8), (1 << 20, 8), (1000, 7)])
def test_split_ranges_uniform_matches_strong_range(n, parts):
    got = u.rs.split_ranges(n, parts)
    assert got == [shard.strong_range(r, parts, n) for r in range(parts)]


@pytest.mark.parametrize("seed,n,parts", [(1, 1000, 2), (2, 65536, 8), (3, 5, 8), (4, 300, 3)])
def test_split_ranges_cost_matches_balanced_ranges(seed, n, parts):
    """Cost-balanced cuts are shard.balanced_ranges' (C3: cost = (k+m)*len)."""
    rng = np.random.default_rng(seed)
    cost = rng.integers(0, 30 * 1250, n)
    assert u.rs.split_ranges(n, parts, cost) == shard.balanced_ranges(cost, parts)


def test_split_ranges_and_set_devices_reject_bad_args():
    from udpspeeder_amd._lib import RsmiError
    with pytest.raises(RsmiError):
        u.rs.split_ranges(10, 0)
    with pytest.raises(RsmiError):
        u.rs.split_ranges(3, 2, [1, -1, 2])
    assert u.lib().rsmi_use_devices(None, -1) != 0
    assert u.lib().rsmi_use_devices(None, 2) != 0
    assert u.rs.get_devices() == []


@pytest.mark.gpu
@pytest.mark.parametrize("devs", [[0], [0, 0], [0, 0, 0]])
def test_multidev_encode_decode_pinned(gpu, oracle, devs):
    """encode_pinned / decode_pinned over the device list: parity equal to the
    oracle's, the decode's rebuilt rows and statuses equal the single-device
    call's, for pinned (zero-copy decode) and pageable (staged) host memory."""
    import torch
    k, n, ln, S, G = 20, 30, 1250, 1280, 3001  # G not a multiple of the device count
    rng = np.random.default_rng(55)
    data = rng.integers(0, 256, (G, k, S), dtype=np.uint8)
    try:
        u.rs.set_devices(devs)
        assert u.rs.get_devices() == devs
        for pinned in (True, False):
            d = torch.from_numpy(data.copy())
            par = torch.zeros((G, n - k, S), dtype=torch.uint8)
            if pinned:
                d, par = d.pin_memory(), par.pin_memory()
            u.rs.encode_pinned(d, par, k, n, ln, chunk_groups=512)
            ref = np.zeros((G, n, S), np.uint8)
            ref[:, :k] = data
            oracle.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G)
            assert np.array_equal(par.numpy()[:, :, :ln], ref[:, k:, :ln]), pinned
            # decode: the whole codeword, 5 random erasures per group, data slots wiped
            full = np.concatenate([data, par.numpy()], axis=1)
            pres = np.ones((G, n), np.uint8)
            for g in range(G):
                pres[g, rng.choice(n, 5, replace=False)] = 0
            h = torch.from_numpy(full.copy())
            h[torch.from_numpy(pres == 0)] = 0xA5
            if pinned:
                h = h.pin_memory()
            st = u.rs.decode_pinned(h, pres, k, n, ln, chunk_groups=700)
            assert (st == 0).all()
            assert np.array_equal(h.numpy()[:, :k, :ln], data[:, :, :ln]), pinned
            path = u.lib().rsmi_last_decode_pinned_path()
            assert path == (1 if pinned else 2), path
    finally:
        u.rs.set_devices([])
    assert u.rs.get_devices() == []


@pytest.mark.gpu
def test_multidev_error_names_the_device(gpu):
    """An invalid device list is rejected and leaves the pool as it was; the
    pool then still runs (an all-zero batch encodes to zero parity)."""
    from udpspeeder_amd._lib import RsmiError
    import torch
    try:
        u.rs.set_devices([0, 0])
        with pytest.raises(RsmiError, match="out of range"):
            u.rs.set_devices([0, 99])
        assert u.rs.get_devices() == [0, 0]  # a rejected list leaves the pool as it was
        d = torch.zeros((64, 4, 256), dtype=torch.uint8)
        p = torch.zeros((64, 2, 256), dtype=torch.uint8)
        u.rs.encode_pinned(d, p, 4, 6, 200)
        assert int(p.sum()) == 0
    finally:
        u.rs.set_devices([])


def _ragged_batch(rng, G, kmax=20):
    ks = rng.integers(1, kmax + 1, G)
    ms = rng.integers(1, 11, G)
    ls = rng.integers(1, 1300, G)
    groups, total = u.make_groups(ks, ks + ms, ls)
    return ks, ms, ls, groups, total


@pytest.mark.gpu
@pytest.mark.parametrize("devs", [[], [0], [0, 0], [0, 0, 0]])
def test_multidev_ragged_pinned(gpu, oracle, devs):
    """rsmi_encode_ragged_pinned / rsmi_decode_ragged_pinned (a mode-0 mix in
    host memory) over the device list, split by summed n*len: parity equal to
    the oracle's for every group, then a non-codeword decode with random
    erasures (some too many) equal to the oracle's rows and statuses."""
    import torch
    from udpspeeder_amd import synth
    rng = np.random.default_rng(len(devs) + 70)
    G = 2501
    ks, ms, ls, groups, total = _ragged_batch(rng, G, kmax=40)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    try:
        u.rs.set_devices(devs)
        h = torch.from_numpy(host.copy()).pin_memory()
        u.rs.encode_ragged_pinned(h, groups, chunk_groups=300)
        exp = host.copy()
        for i in range(G):
            d = groups[i]
            seg = exp[d.offset:d.offset + d.n * d.shard_stride]
            oracle.encode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1)
            exp[d.offset:d.offset + d.n * d.shard_stride] = seg
            got = h.numpy()[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
            assert np.array_equal(got[:, :d.len], seg.reshape(d.n, d.shard_stride)[:, :d.len]), i
        # decode a non-codeword batch: every group's own (k, n, len), erasures up to m + 1
        flags = np.zeros((G, 256), np.uint8)
        for i in range(G):
            n = int(ks[i] + ms[i])
            flags[i, :n] = 1
            flags[i, rng.choice(n, min(int(rng.integers(0, ms[i] + 2)), n), replace=False)] = 0
        h2 = torch.from_numpy(host.copy()).pin_memory()
        st = u.rs.decode_ragged_pinned(h2, groups, synth.present_bits(flags), chunk_groups=257)
        for i in range(G):
            d = groups[i]
            seg = host[d.offset:d.offset + d.n * d.shard_stride].copy()
            ost = oracle.decode_batch(d.k, d.n, seg, 0, d.shard_stride, d.len, 1, flags[i:i + 1, :d.n])
            assert st[i] == ost[0], i
            if st[i] == 0:
                got = h2.numpy()[d.offset:d.offset + d.k * d.shard_stride].reshape(d.k, d.shard_stride)
                assert np.array_equal(got[:, :d.len], seg.reshape(d.n, d.shard_stride)[:d.k, :d.len]), i
    finally:
        u.rs.set_devices([])


def test_ragged_pinned_rejects_unordered_groups():
    """The host ragged entries need ascending, non-overlapping group spans
    (each chunk is one contiguous copy); checked before any GPU work."""
    from udpspeeder_amd._lib import RsmiError
    groups, total = u.make_groups([2, 3], [4, 5], [100, 100])
    groups[0].offset, groups[1].offset = groups[1].offset, groups[0].offset
    host = np.zeros(total + 64, np.uint8)
    with pytest.raises(RsmiError, match="ascending"):
        u.rs.encode_ragged_pinned(host, groups)


@pytest.mark.gpu
def test_multidev_set_devices_during_calls(gpu, oracle):
    """rsmi_use_devices racing split calls from another thread: every call
    either runs on the list it saw or on the current device -- never a silent
    no-op (run_split decides under its lock) -- and its parity is
    right either way."""
    import threading
    import torch
    k, n, ln, S, G = 10, 14, 400, 400, 777
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, (G, k, S), dtype=np.uint8)
    ref = np.zeros((G, n, S), np.uint8)
    ref[:, :k] = data
    oracle.encode_batch(k, n, ref.reshape(-1), n * S, S, ln, G)
    stop = threading.Event()
    errs = []

    def flip():
        i = 0
        while not stop.is_set():
            try:
                u.rs.set_devices([0, 0] if i % 2 == 0 else [])
            except Exception as e:  # noqa: BLE001
                errs.append(e)
            i += 1

    th = threading.Thread(target=flip)
    th.start()
    try:
        d = torch.from_numpy(data).pin_memory()
        for _ in range(30):
            par = torch.zeros((G, n - k, S), dtype=torch.uint8).pin_memory()
            u.rs.encode_pinned(d, par, k, n, ln, chunk_groups=128)
            assert np.array_equal(par.numpy()[:, :, :ln], ref[:, k:, :ln])
    finally:
        stop.set()
        th.join()
        u.rs.set_devices([])
    assert not errs
