"""Batch decode keeps unpackPacked's all-or-nothing contract per unit
(message.zig:88-145: `unpackPacked` sizes the input with estimateUnpackedSize and
returns UnexpectedEof / no output before it writes a byte): a mid or long unit whose
status is UNEXPECTED_EOF or OUT_OF_SPACE leaves its output slot exactly as it was.
Small units (<= 512 packed bytes into <= 8-KiB slots, decoded a lane each in one
streaming pass) and, under the streaming mid-unit decoder, mid units are
the documented exception: a failed one may hold a prefix of its output,
never a byte past its out_cap; with capnp_packed_set_all_or_nothing(1) they are
all-or-nothing too (the group-staged small decoder, the two-pass mid decoder).

Units of each size class are decoded from a dense packed stream
(unaligned unit starts) into slots pre-filled with a sentinel byte:
- every third unit is its packed bytes less the last one (a cut record: EOF at the very
  end of the unit, after the decoder has seen everything else),
- every fifth unit gets a slot 8 B short of its decoded size (OUT_OF_SPACE),
- the rest decode normally and must match the oracle (message.zig:88-145).
Statuses are compared with the oracle (tests/oracle.py) unit by unit.
"""
import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


DEV = "cuda"
SENTINEL = 0xA5

# (class, words per unit, zero-byte threshold): small units are <= 512 packed bytes into
# slots <= 8 KiB (a lane each), mid units the indexed two-pass decoder, long units
# (> 5120 packed bytes) the window-parallel decoder
CLASSES = [("small", 32, 128), ("mid", 512, 128), ("long", 1024, 26)]


def words(rng, n_words, thr):
    b = rng.integers(1, 256, n_words * 8, dtype=np.uint8)
    b[rng.integers(0, 256, n_words * 8) < thr] = 0
    return b.tobytes()


@pytest.mark.parametrize("cls,n_words,thr", CLASSES, ids=[c[0] for c in CLASSES])
def test_failed_units_leave_their_slot_untouched(cls, n_words, thr, decoder):
    check_class(cls, n_words, thr, strict=False, prefix_mid=decoder == "words")


@pytest.mark.parametrize("dec", ["words", "auto"])
@pytest.mark.parametrize("cls,n_words,thr", CLASSES[1:], ids=[c[0] for c in CLASSES[1:]])
def test_mid_units_all_or_nothing_when_asked_under_stream(cls, n_words, thr, dec):
    """capnp_packed_set_all_or_nothing(1) routes mid units past the single-read words decoder
    (which may leave a failed unit's prefix), forced or by the default's rule, to the two-pass
    decoder: every failed slot untouched."""
    if not cp.decoder_available(dec):
        pytest.skip(f"the {dec} decoder is not in this build")
    prev = cp.set_all_or_nothing(True)
    try:
        with cp.decoder(dec):
            check_class(cls, n_words, thr, strict=True)
    finally:
        cp.set_all_or_nothing(prev)


def test_small_units_all_or_nothing_when_asked():
    prev = cp.set_all_or_nothing(True)
    try:
        check_class("small", 32, 128, strict=True)
        check_class("small", 16, 230, strict=True)
    finally:
        cp.set_all_or_nothing(prev)


def check_class(cls, n_words, thr, strict, prefix_mid=False):
    rng = np.random.default_rng(0xC0DE + n_words)
    n = 384
    data = [words(rng, n_words, thr) for _ in range(n)]
    packed = []
    for i, d in enumerate(data):
        st, p = oracle.pack(d)
        assert st == oracle.OK
        packed.append(p[:-1] if i % 3 == 1 else p)
    caps = [len(d) - 8 if i % 5 == 2 else len(d) for i, d in enumerate(data)]
    if cls == "long":
        assert min(len(p) for p in packed) > 5120
    if cls == "small":
        assert max(len(p) for p in packed) <= 512

    plen = np.array([len(p) for p in packed], dtype=np.int64)
    poff = np.zeros(n, dtype=np.int64)
    poff[1:] = np.cumsum(plen)[:-1]
    cap = np.array(caps, dtype=np.int64)
    slot = (np.array([len(d) for d in data], dtype=np.int64) + 63) // 64 * 64
    ooff = np.zeros(n, dtype=np.int64)
    ooff[1:] = np.cumsum(slot)[:-1]

    d_in = torch.from_numpy(np.frombuffer(b"".join(packed), dtype=np.uint8).copy()).to(DEV)
    d_out = torch.full((int(slot.sum()),), SENTINEL, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    t = lambda a: torch.from_numpy(a).to(DEV)
    cp.decode_batch(d_in, t(poff), t(plen), d_out, t(ooff), t(cap), out_len, status)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    st = status.cpu().numpy()
    ol = out_len.cpu().numpy()

    seen = set()
    for i in range(n):
        ost, ref = oracle.unpack(packed[i])
        want = ost if ost != oracle.OK or len(ref) <= caps[i] else oracle.OUT_OF_SPACE
        assert st[i] == want, (cls, i, st[i], want)
        seen.add(int(want))
        s = out[ooff[i]:ooff[i] + slot[i]]
        if want == oracle.OK:
            assert ol[i] == len(ref)
            assert s[:len(ref)].tobytes() == ref, (cls, i)
            assert (s[len(ref):] == SENTINEL).all(), (cls, i, "bytes past out_len written")
        elif (cls == "small" or (cls == "mid" and prefix_mid)) and not strict:
            assert (s[caps[i]:] == SENTINEL).all(), (cls, i, int(want), "bytes past out_cap written")
        else:
            assert (s == SENTINEL).all(), (cls, i, int(want), "failed unit wrote into its slot")
    assert seen == {oracle.OK, oracle.UNEXPECTED_EOF, oracle.OUT_OF_SPACE}
