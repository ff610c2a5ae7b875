"""The parity packets cooked in the encoder's epilogue (RSMI_OPT_PARITY_COOK,
rsmi_internal.hpp EpiRec): a fused cooked FEC run gives the same cooked bytes
and lengths with the option on as with it off -- the off path is the one
pinned to the reference's do_cook elsewhere (test_fec_frame.py) -- and the
epilogue really ran for the codes that have a split-k network.  Every
cooked packet also de-cooks through the oracle to the plain packet of the
restated manager (oracle/fec_frame.py)."""
import numpy as np
import pytest

from oracle.cpu import cook_payloads
from oracle.fec_frame import EncodeManager

pytestmark = pytest.mark.gpu


def _stream(seed, n, lmax):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, lmax + 1, n).astype(np.int32)
    lens[rng.random(n) < 0.01] = -1  # timer flushes
    pay = cook_payloads(seed, 0, n, np.maximum(lens, 0), lmax)
    return lens, [None if lens[i] < 0 else pay[i, :lens[i]].tobytes() for i in range(n)]


def _run(torch, rs, mode, lens, ev, cuts, key, flags, on, stride_extra=0):
    import udpspeeder_amd as u
    from udpspeeder_amd._lib import RSMI_OPT_PARITY_COOK
    from udpspeeder_amd.cook import CookContext
    from udpspeeder_amd.fec import FecEncoder
    prev = u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, 1 if on else 0)
    try:
        enc = FecEncoder(rs, mode, 1250, 200, seq0=0xFFFFFF00)
        ctx = CookContext(key, flags)
        pk, used = [], 0
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
            S = FecEncoder.slot_stride_for(max(p.slot_stride_min - 128, 0)) + stride_extra
            slots = torch.full((max(1, p.n_slots) * S,), 0xEE, dtype=torch.uint8, device="cuda")
            out = torch.full((max(1, p.n_slots) * S,), 0x5A, dtype=torch.uint8, device="cuda")
            ol = enc.run_cooked(slots, S, ctx, 77 + bi, out=out)
            torch.cuda.synchronize()
            used += enc.last_parity_cooked()
            ol = ol.cpu().numpy()[:len(p.packets)]
            h = out.cpu().numpy()
            pk += [(h[s * S + 120:s * S + 120 + int(l)].tobytes(), int(l)) for (s, _, _), l in zip(p.packets, ol)]
            del inbuf
        enc.close()
        ctx.close()
        return pk, used
    finally:
        u.lib().rsmi_option(RSMI_OPT_PARITY_COOK, prev)


@pytest.mark.parametrize("rs,mode,lmax,flags,key", [
    ("20:10", 0, 1200, 0, b"secret key"),
    ("20:10", 1, 1250, 0, b"k"),
    ("1:3,2:4,10:6,20:10", 0, 700, 0, b"another key"),
    ("1:3,2:4,10:6,20:10", 1, 900, 0, b"another key"),
    ("20:10", 1, 1250, 4, b"unused"),   # no XOR stage: the zero key stream
    ("20:10", 1, 1250, 2, b"key2"),     # no obscure stage: iv_len 0
    ("20:10", 1, 1250, 1, b"key3"),     # no checksum
    ("10:5,20:10", 1, 1000, 0, b""),    # empty key
])
def test_parity_cook_same_bytes(gpu, cook_oracle, rs, mode, lmax, flags, key):
    import torch
    n = 6000
    lens, ev = _stream(0xC0DE + lmax + mode + flags, n, lmax)
    cuts = np.array([0, 2500, 2501, n])
    off, used_off = _run(torch, rs, mode, lens, ev, cuts, key, flags, False)
    on, used_on = _run(torch, rs, mode, lens, ev, cuts, key, flags, True)
    assert used_off == 0
    if "20:10" in rs:
        assert used_on > 0, "the epilogue did not run"
    assert [l for _, l in on] == [l for _, l in off]
    bad = [i for i, (a, b) in enumerate(zip(on, off)) if a[0] != b[0]]
    assert not bad, (len(bad), bad[:5])
    # and the cooked bytes de-cook to the restated manager's packets
    em = EncodeManager(rs, mode, 1250, 200, 0xFFFFFF00)
    exp = []
    for e in ev:
        em.input(e)
        exp += em.output()
    assert len(exp) == len(on)
    for i in range(0, len(on), 37):
        rc, b, nl = cook_oracle.de_cook(on[i][0], key, flags)
        assert rc == 0 and b[:nl] == exp[i], i


def test_parity_cook_larger_slots(gpu):
    """A slot stride well past the minimum (line padding columns past the
    payload are encoded too, and land in the output as plain bytes past the
    cooked packet)."""
    import torch
    lens, ev = _stream(0xBEEF, 3000, 1250)
    cuts = np.array([0, 3000])
    off, _ = _run(torch, "20:10", 1, lens, ev, cuts, b"key", 0, False, stride_extra=512)
    on, used = _run(torch, "20:10", 1, lens, ev, cuts, b"key", 0, True, stride_extra=512)
    assert used > 0
    assert on == off
