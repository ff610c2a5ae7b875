"""GPU parity of the reference-placement decode (rsmi_decode_dev_ref): every
rebuilt data row lands in the parity survivor's buffer that fec_decode's shuffle
moves into data[i] (lib/fec.cpp:755-788, 872-877), and the slot map equals the
pointer permutation rs_decode leaves in data[0..k-1] -- checked against the
reference's own permutations (decode_small.npz ptr_out), the oracle's
per-group pointer dance, and the full-size C2 non-codeword digest."""
import hashlib
import os

import numpy as np
import pytest

from oracle.cpu import DATA_SEED, group_data

pytestmark = pytest.mark.gpu


def stride_for(ln):
    return max(16, (ln + 15) // 16 * 16)


def pad_end(ln, stride):
    return min(stride, (ln + 127) // 128 * 128)


def upload(buf, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(buf)).to(device)


def _decode_cases():
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "decode_small.npz"))
    return sorted({k.split("__")[0] for k in d.files})


def _ref_decode(u, t, pres_t, k, n, ln, fused=True):
    import torch
    G = t.shape[0]
    smap = torch.full((G, k), 0xEE, dtype=torch.uint8, device=t.device)
    prev = u.rs.set_fused_decode(fused)
    try:
        st = u.decode(t, pres_t, k, n, ln, placement="reference", slot_map=smap)
    finally:
        u.rs.set_fused_decode(prev)
    return st, smap


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", _decode_cases())
def test_ref_placement_small_golden(gpu, golden, name, fused):
    """Every decode_small case: data rows read through the slot map hash to the
    reference's data_out digest, and group 0's map is the reference's ptr_out."""
    import udpspeeder_amd as u
    D = golden.dec
    k, n, ln, ng, codeword = [int(x) for x in D[f"{name}__meta"]]
    present = D[f"{name}__present"]
    S = stride_for(ln)
    buf = np.zeros((ng, n, S), np.uint8)
    buf[:, :k, :ln] = group_data(DATA_SEED, 0, ng, k, ln)
    if codeword:
        u.encode(t0 := upload(buf, gpu), k, n, ln)
        buf = t0.cpu().numpy()
    else:
        buf[:, k:, :ln] = group_data(DATA_SEED ^ 0xFFFF, 0, ng, n - k, ln)
    buf[present == 0] = 0xA5
    t = upload(buf, gpu)
    st, smap = _ref_decode(u, t, upload(present, gpu), k, n, ln, fused)
    st = st.cpu().numpy()
    assert (st == D[f"{name}__status"]).all()
    m = smap.cpu().numpy()
    po = D[f"{name}__ptr_out"][:k]
    assert (m[0].astype(np.int64) == np.where(po < 0, 255, po)).all()
    for g in range(ng):
        assert (m[g] == u.ref_slot_map(k, n, present[g])).all()
    out = t.cpu().numpy()
    if (st == 0).all():
        rows = np.stack([out[g, m[g].astype(np.int64), :ln] for g in range(ng)])
        assert hashlib.sha256(rows.tobytes()).hexdigest() == D[f"{name}__data_out_sha"].tobytes().hex()
    # slots no row was moved into are the input bytes (erased data slots are
    # scratch)
    for g in range(ng):
        if st[g] != 0:
            assert (out[g] == buf[g]).all()
            continue
        dst = set(int(x) for x in m[g]) - set(range(k))
        for j in range(n):
            if j in dst or (j < k and not present[g, j]):
                continue
            assert (out[g, j] == buf[g, j]).all(), (g, j)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("k,n,ln,ner", [(20, 30, 1250, 5), (20, 30, 1250, 10), (7, 13, 999, 6),
                                        (1, 4, 77, 3), (64, 128, 48, 64), (3, 6, 3, 3),
                                        (10, 16, 4096, 6), (2, 255, 20, 253), (20, 30, 3000, 8)])
def test_ref_placement_vs_oracle_pointers(gpu, oracle, k, n, ln, ner, fused):
    """Random non-codeword groups: the bytes behind each data[i] and the
    permutation equal the oracle's rs_decode pointer dance, group by group."""
    import udpspeeder_amd as u
    G = 29
    S = stride_for(ln)
    rng = np.random.default_rng(k * 7 + n + ln)
    buf = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    present = np.ones((G, n), np.uint8)
    for g in range(G):
        present[g, rng.choice(n, min(int(rng.integers(0, ner + 2)), n), replace=False)] = 0
    t = upload(buf, gpu)
    st, smap = _ref_decode(u, t, upload(present, gpu), k, n, ln, fused)
    st = st.cpu().numpy()
    m = smap.cpu().numpy()
    out = t.cpu().numpy()
    for g in range(G):
        shards = [bytes(buf[g, j, :ln]) if present[g, j] else None for j in range(n)]
        rc, perm, after = oracle.decode_ptrs(k, n, shards, ln)
        assert st[g] == rc, g
        if rc != 0:
            continue
        for i in range(k):
            assert m[g, i] == perm[i], (g, i)
            assert out[g, m[g, i], :ln].tobytes() == after[perm[i]][:ln], (g, i)
        # nothing past the slot padding is written
        pad = pad_end(ln, S)
        assert (out[g, :, pad:] == buf[g, :, pad:]).all()


def test_ref_placement_c2_full_noncodeword_sha(gpu, golden):
    """C2 at full size: rows read through the device slot map hash to the
    reference's digest, and the map equals the host closed form."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    F = golden.full["c2_decode_noncodeword"]
    k, n, ln, G = F["k"], F["n"], F["len"], F["groups"]
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, DATA_SEED)
    u.fill_data(t[:, k:], n - k, ln, F["parity_seed"])
    pres = synth.erasure_present(F["erase_seed"], 0, G, n, F["erasures"])
    smap = torch.empty((G, k), dtype=torch.uint8, device=gpu)
    st = u.decode(t, upload(pres, gpu), k, n, ln, placement="reference", slot_map=smap)
    assert int((st != 0).sum().item()) == 0
    h = hashlib.sha256()
    for g0 in range(0, G, 8192):
        rows = u.reference_rows(t[g0:g0 + 8192], smap[g0:g0 + 8192])
        h.update(np.ascontiguousarray(rows[:, :, :ln].cpu().numpy()).tobytes())
    assert h.hexdigest() == F["data_out_sha256"]
    m = smap.cpu().numpy()
    for g in range(0, G, 4099):
        assert (m[g] == u.ref_slot_map(k, n, pres[g])).all()


def test_ref_placement_roundtrip_repeated(gpu):
    """The bench's step: encode then reference-placement decode, repeated on
    one buffer -- each encode restores the parity the previous decode wrote
    over, so every decode sees the codeword and returns the data."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 1250, 16384
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, 77)
    orig = t[:, :k, :ln].clone()
    pres = upload(synth.erasure_present(5, 0, G, n, 5), gpu)
    smap = torch.empty((G, k), dtype=torch.uint8, device=gpu)
    for _ in range(3):
        u.encode(t, k, n, ln)
        st = u.decode(t, pres, k, n, ln, placement="reference", slot_map=smap)
        assert int((st != 0).sum().item()) == 0
        assert torch.equal(u.reference_rows(t, smap)[:, :, :ln], orig)


# ---------------------------------------------------------------- ragged
def _ragged_ref_check(u, oracle, groups, host, flags, out, st, smap, stride):
    """Every group against the oracle: status, the slot map (host closed form,
    entries < stride), the bytes behind each data[i], and every slot that is
    neither a destination nor an erased data slot left as it was."""
    for i in range(len(groups)):
        d = groups[i]
        n, k, S = d.n, d.k, d.shard_stride
        seg = host[d.offset:d.offset + n * S].copy()
        ost = oracle.decode_batch(k, n, seg, 0, S, d.len, 1, flags[i:i + 1, :n])
        assert st[i] == ost[0], (i, k, n)
        if st[i] not in (0, -1):
            continue
        exp_map = u.ref_slot_map(k, n, flags[i, :n])
        kk = min(k, stride)
        assert (smap[i, :kk] == exp_map[:kk]).all(), (i, k, n)
        got = out[d.offset:d.offset + n * S].reshape(n, S)
        org = host[d.offset:d.offset + n * S].reshape(n, S)
        if st[i] == 0:
            exp = seg.reshape(n, S)
            for j in range(k):
                assert (got[exp_map[j], :d.len] == exp[j, :d.len]).all(), (i, k, n, j)
        dst = set(int(x) for x in exp_map) - set(range(k)) if st[i] == 0 else set()
        for j in range(n):
            if j in dst or (j < k and not flags[i, j]):
                continue
            assert (got[j] == org[j]).all(), (i, j)
        pad = pad_end(d.len, S)
        assert (got[:, pad:] == org[:, pad:]).all(), i


@pytest.mark.parametrize("form,kmax,stride", [("plan", 60, 48), ("dev", 60, 48), ("plan", 200, 200),
                                               ("dev", 200, 160)])
def test_ref_ragged_many_codes_vs_oracle(gpu, oracle, form, kmax, stride):
    """Ragged reference-placement decode over ~200 codes: e up to 10 (row
    blocks of 5: the earlier blocks parked and moved), k up to 60 (k > 32:
    the workgroup kernel) or 200 (k > 64, too-few groups among them: their
    map entries past 64), lengths 1..3000 (several tiles), too-few groups;
    slot maps with a stride smaller than some k."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    rng = np.random.default_rng(606 + kmax)
    G = 500 if kmax <= 60 else 160
    ks = rng.integers(1, kmax + 1, G)
    ms = rng.integers(1, 21, G)
    ms = np.minimum(ms, 256 - ks)
    ls = rng.integers(1, 3000 if kmax <= 60 else 700, G)
    ls[:4] = [1, 16, 1280, 1281]
    groups, total = u.make_groups(ks, ks + ms, ls)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    flags = np.zeros((G, 256), np.uint8)
    for i in range(G):
        n, m = int(ks[i] + ms[i]), int(ms[i])
        flags[i, :n] = 1
        flags[i, rng.choice(n, min(int(rng.integers(0, 12)), n), replace=False)] = 0
    for c in set(zip(ks.tolist(), (ks + ms).tolist())):
        u.prepare_code(*c)
    base = upload(host, gpu)
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    smap = torch.full((G, stride), 0xEE, dtype=torch.uint8, device=gpu)
    if form == "plan":
        plan = u.rs.RaggedPlan(groups, wait_codes=False)
        st = plan.decode(base, bits, placement="reference", slot_map=smap)
        torch.cuda.synchronize()
        plan.close()
    else:
        from udpspeeder_amd._lib import check
        st = torch.empty(G, dtype=torch.int32, device=gpu)
        dg = u.rs.groups_to_device(groups, gpu)
        check(u.lib().rsmi_decode_ragged_dev_ref(dg.data_ptr(), G, base.data_ptr(), bits.data_ptr(),
                                                 st.data_ptr(), kmax, smap.data_ptr(), stride, None),
              "rsmi_decode_ragged_dev_ref")
    _ragged_ref_check(u, oracle, groups, host, flags, base.cpu().numpy(), st.cpu().numpy(),
                      smap.cpu().numpy(), stride)


def test_ref_ragged_c3_full_sha(gpu, golden):
    """C3 decode at full size through a plan with the reference's placement:
    the rows read through the slot map hash to the reference's digest."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    F = golden.full["c3_ragged_decode"]
    table = u.rs_from_str(F["fec"])
    ks, ms, ls = synth.ragged_mix(F["ragged_seed"], 0, F["groups"], [y for _, y in table])
    groups, total = u.make_groups(ks, ks + ms, ls)
    base = torch.zeros(total, dtype=torch.uint8, device=gpu)
    u.rs.fill_ragged(base, u.rs.groups_to_device(groups, gpu), len(groups), DATA_SEED)
    par, _ = u.make_groups(np.maximum(ms, 1), np.maximum(ms, 1), ls)
    for i in range(len(groups)):
        par[i].offset = groups[i].offset + groups[i].k * groups[i].shard_stride
        par[i].shard_stride = groups[i].shard_stride
    u.rs.fill_ragged(base, u.rs.groups_to_device(par, gpu), len(groups), F["parity_seed"])
    flags = synth.ragged_erasures(F["erase_seed"], 0, ks + ms, ms, F["erasures"])
    bits = torch.from_numpy(synth.present_bits(flags).view(np.int32)).to(gpu)
    plan = u.rs.RaggedPlan(groups)
    G = len(groups)
    smap = torch.empty((G, 20), dtype=torch.uint8, device=gpu)
    st = plan.decode(base, bits, placement="reference", slot_map=smap)
    torch.cuda.synchronize()
    plan.close()
    assert int((st != 0).sum()) == 0
    out = base.cpu().numpy()
    m = smap.cpu().numpy()
    h = hashlib.sha256()
    for i in range(G):
        d = groups[i]
        rows = out[d.offset:d.offset + d.n * d.shard_stride].reshape(d.n, d.shard_stride)
        h.update(rows[m[i, :d.k].astype(np.int64), :d.len].tobytes())
    assert h.hexdigest() == F["data_out_sha256"]


def test_ref_placement_graph_capture_replay(gpu, oracle):
    """The headline step (encode, then the reference-placement decode with its
    slot map) captured in a hipGraph: each replay recomputes from the current
    data, the rows read through the map equal the data, and the map equals the
    host closed form (the present flags are fixed)."""
    import torch
    import udpspeeder_amd as u
    from udpspeeder_amd import synth
    k, n, ln, G = 20, 30, 1250, 777
    t = torch.zeros((G, n, 1280), dtype=torch.uint8, device=gpu)
    pres_h = synth.erasure_present(4, 0, G, n, 5)
    pres = upload(pres_h, gpu)
    st = torch.empty(G, dtype=torch.int32, device=gpu)
    sm = torch.empty((G, k), dtype=torch.uint8, device=gpu)
    u.fill_data(t, k, ln, 1)
    u.reserve(k, n, G)
    u.encode(t, k, n, ln)
    u.decode(t, pres, k, n, ln, status=st, placement="reference", slot_map=sm)  # warm-up
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        u.encode(t, k, n, ln)
        u.decode(t, pres, k, n, ln, status=st, placement="reference", slot_map=sm)
    for seed in (2, 3):
        u.fill_data(t, k, ln, seed)
        sm.fill_(0xEE)
        g.replay()
        torch.cuda.synchronize()
        assert int((st != 0).sum()) == 0
        assert torch.equal(u.reference_rows(t, sm)[:, :, :ln], t[:, :k, :ln])
        m = sm.cpu().numpy()
        for gi in range(0, G, 37):
            assert (m[gi] == u.ref_slot_map(k, n, pres_h[gi])).all()
