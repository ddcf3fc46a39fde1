"""Randomised mixed-class stress of the batch codec against the oracle (message.zig:88-271),
every unit compared: units of every size class (small / mid / long / huge) and density in
one batch, with truncated packed units, short output slots, misaligned output slots and
empty units mixed in, decoded from a dense packed stream at unaligned offsets into slots
with canary bytes around them, under each mid-unit decoder and both small-unit modes
(capnp_packed_set_decoder / capnp_packed_set_all_or_nothing). Checks per unit: status,
out_len, bytes, and that nothing outside a slot changes (and, where the contract says so,
nothing inside a failed unit's slot). Also the size batch (estimateUnpackedSize) and the
encode batch on the same units."""
import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
CANARY = 0x5A


def unit_bytes(rng, i):
    kind = i % 10
    if kind < 5:
        nw = int(rng.integers(0, 80))           # small
    elif kind < 8:
        nw = int(rng.integers(80, 700))         # mid
    elif kind < 9:
        nw = int(rng.integers(700, 12000))      # long
    else:
        nw = int(rng.integers(12000, 40000)) if rng.random() < 0.3 else int(rng.integers(0, 4))
    thr = int(rng.choice([0, 26, 128, 230, 250, 256]))
    b = rng.integers(1, 256, nw * 8, dtype=np.uint8)
    b[rng.integers(0, 256, nw * 8) < thr] = 0
    return b.tobytes()


def build(seed, n):
    rng = np.random.default_rng(seed)
    data = [unit_bytes(rng, i) for i in range(n)]
    packed, caps, flags = [], [], []
    for i, d in enumerate(data):
        st, p = oracle.pack(d)
        assert st == oracle.OK
        r = rng.random()
        if r < 0.08 and len(p) > 1:
            p = p[:-int(rng.integers(1, min(len(p), 12)))]  # cut: EOF, or a shorter valid stream
            flags.append("cut")
        else:
            flags.append("")
        cap = len(d)
        if rng.random() < 0.08 and cap >= 8:
            cap -= 8 * int(rng.integers(1, max(2, cap // 8)))  # short slot
        caps.append(max(cap, 0))
        packed.append(p)
    return rng, data, packed, caps, flags


def run_decode(rng, packed, caps, misalign_every=37):
    n = len(packed)
    poff, pos = [], 0
    for p in packed:
        pos += int(rng.integers(0, 16))
        poff.append(pos)
        pos += len(p)
    blob = np.zeros(pos + 16, dtype=np.uint8)
    for i, p in enumerate(packed):
        blob[poff[i]:poff[i] + len(p)] = np.frombuffer(p, dtype=np.uint8)
    ooff, o = [], 0
    for i, c in enumerate(caps):
        o += 16 + (8 * int(rng.integers(0, 4)))
        ooff.append(o + (3 if i % misalign_every == 5 else 0))  # a misaligned slot now and then
        o += c + 16
    out = torch.full((o + 32,), CANARY, dtype=torch.uint8, device=DEV)
    t = lambda a: torch.tensor(a, dtype=torch.int64, device=DEV)  # noqa: E731
    d_in = torch.from_numpy(blob).to(DEV)
    out_len = torch.full((n,), -1, dtype=torch.int64, device=DEV)
    st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_in, t(poff), t([len(p) for p in packed]), out, t(ooff), t(caps), out_len, st)
    sz_len = torch.full((n,), -1, dtype=torch.int64, device=DEV)
    sz_st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decoded_size_batch(d_in, t(poff), t([len(p) for p in packed]), sz_len, sz_st)
    torch.cuda.synchronize()
    return (ooff, out.cpu().numpy(), out_len.cpu().numpy(), st.cpu().numpy(), sz_len.cpu().numpy(), sz_st.cpu().numpy(),
            poff)


def check(packed, caps, ooff, out, out_len, st, sz_len, sz_st, poff, strict_small, prefix_mid=False):
    covered = np.zeros(out.size, dtype=bool)
    for i, p in enumerate(packed):
        es, ref = oracle.unpack(p)
        ss, sn = oracle.decoded_size(p)
        assert (int(sz_st[i]), int(sz_len[i])) == (ss, sn if ss == 0 else 0), ("size", i)
        slot = out[ooff[i]:ooff[i] + caps[i]]
        covered[ooff[i]:ooff[i] + caps[i]] = True
        if ooff[i] % 8:
            want = oracle.INVALID_ARGUMENT if len(p) else oracle.OK  # an empty unit writes nothing
            assert int(st[i]) == want, ("misaligned", i, int(st[i]))
            assert (slot == CANARY).all()
            continue
        want = es if es != oracle.OK or len(ref) <= caps[i] else oracle.OUT_OF_SPACE
        assert int(st[i]) == want, (i, len(p), caps[i], int(st[i]), want)
        if want == oracle.OK:
            assert int(out_len[i]) == len(ref) and slot[:len(ref)].tobytes() == ref, i
            assert (slot[len(ref):] == CANARY).all(), i
        else:
            if want == oracle.OUT_OF_SPACE:
                assert int(out_len[i]) == len(ref), i
            small = len(p) <= 512 and caps[i] <= 8192
            # the streaming and words mid decoders may leave a prefix too; long units
            # (> 320 packed 16-B pieces from the unit's 16-B aligned base) never do
            mid = not small and (poff[i] % 16 + len(p) + 15) // 16 <= 320
            if strict_small or not (small or (prefix_mid and mid)):
                assert (slot == CANARY).all(), ("failed unit wrote into its slot", i, int(want))
    assert (out[~covered] == CANARY).all(), "bytes outside every slot changed"


@pytest.mark.parametrize("strict", [False, True])
def test_mixed_class_stress(decoder, strict):
    seed = 0xC0DE5000 + {"twopass": 0, "words": 6}[decoder] + strict
    rng, data, packed, caps, _ = build(seed, 1500)
    prev = cp.set_all_or_nothing(strict)
    try:
        res = run_decode(rng, packed, caps)
    finally:
        cp.set_all_or_nothing(prev)
    check(packed, caps, *res, strict_small=strict, prefix_mid=decoder == "words" and not strict)


def test_encode_batch_stress():
    rng, data, _, _, _ = build(0xC0DE5100, 1500)
    n = len(data)
    ioff, pos = [], 0
    for d in data:
        ioff.append(pos)
        pos += len(d)
    blob = np.frombuffer(b"".join(data) or b"\0", dtype=np.uint8).copy()
    caps = [cp.encode_bound(len(d)) if rng.random() > 0.1 else max(0, len(oracle.pack(d)[1]) - 1) for d in data]
    ooff, o = [], 0
    for c in caps:
        o += 16 + int(rng.integers(0, 16))
        ooff.append(o)
        o += c + 16
    out = torch.full((o + 32,), CANARY, dtype=torch.uint8, device=DEV)
    t = lambda a: torch.tensor(a, dtype=torch.int64, device=DEV)  # noqa: E731
    plen = torch.full((n,), -1, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(torch.from_numpy(blob).to(DEV), t(ioff), t([len(d) for d in data]), out, t(ooff), t(caps),
                    plen, pst)
    torch.cuda.synchronize()
    out, plen, pst = out.cpu().numpy(), plen.cpu().numpy(), pst.cpu().numpy()
    covered = np.zeros(out.size, dtype=bool)
    for i, d in enumerate(data):
        _, exp = oracle.pack(d)
        covered[ooff[i]:ooff[i] + caps[i]] = True
        if len(exp) <= caps[i]:
            assert (int(pst[i]), int(plen[i])) == (0, len(exp)), i
            assert out[ooff[i]:ooff[i] + len(exp)].tobytes() == exp, i
        else:
            assert (int(pst[i]), int(plen[i])) == (cp.OUT_OF_SPACE, len(exp)), i
    assert (out[~covered] == CANARY).all()
