"""Message.validate on the device (capnp_packed_validate_batch, message.zig:699-969)
against the CPU oracle (oracle_validate), bit-exact in status and traversal words:

- the reference's known-answer tests (message_test.zig:184-260), through the batch
  call and through the host mirror Message.validate;
- large corpora of random message trees with every pointer encoding, mostly damaged,
  at byte-unaligned offsets in one device buffer, under several limit sets;
- the reference's malformed-buffer fuzz shape (message_test.zig:1057-1093), raw and
  after unpackPacked;
- nesting at the device stack's depth (64), wide pointer lists, big data lists, and
  argument errors;
- the reference's real messages (tests/golden/fixtures: capnp testdata `binary` and
  `segmented`, interop `fixture_single` / `fixture_far`, and the unpacked forms of their
  packed twins) under default and tight limits;
- nesting limits above 64 (the deep pass: frames in global memory), up to 2^32 - 1.
"""
import os
import numpy as np
import pytest

import capnp_packed as cp
import msggen
import oracle
from validate_cases import CODES, KATS, NAMES, kat_options

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


def run_batch(msgs, pad_seed=None, **opts):
    """Validate a list of framed messages in one batch; returns (status, words) arrays."""
    rng = np.random.default_rng(pad_seed) if pad_seed is not None else None
    offs, parts, pos = [], [], 0
    for m in msgs:
        if rng is not None:  # byte-unaligned starts
            gap = int(rng.integers(0, 8))
            parts.append(b"\xAA" * gap)
            pos += gap
        offs.append(pos)
        parts.append(m)
        pos += len(m)
    blob = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8)
    d_in = torch.from_numpy(blob.copy()).to(DEV)
    in_off = torch.tensor(offs, dtype=torch.int64, device=DEV)
    in_len = torch.tensor([len(m) for m in msgs], dtype=torch.int64, device=DEV)
    st = torch.full((len(msgs),), -1, dtype=torch.int32, device=DEV)
    words = torch.full((len(msgs),), -1, dtype=torch.int64, device=DEV)
    cp.validate_batch(d_in, in_off, in_len, st, words, **opts)
    torch.cuda.synchronize()
    return st.cpu().numpy(), words.cpu().numpy()


def check_against_oracle(msgs, opts, pad_seed=None):
    st, words = run_batch(msgs, pad_seed=pad_seed, **opts)
    seen = set()
    for i, m in enumerate(msgs):
        exp = oracle.validate(m, **opts)
        assert (int(st[i]), int(words[i])) == exp, \
            f"message {i} ({len(m)} B, {opts}): device {(NAMES.get(int(st[i])), int(words[i]))} " \
            f"oracle {(NAMES[exp[0]], exp[1])}"
        seen.add(exp[0])
    return seen


@pytest.mark.parametrize("name,build,opts,expected", KATS, ids=[k[0] for k in KATS])
def test_reference_kats_batch(name, build, opts, expected):
    o = kat_options(opts)
    st, words = run_batch([build()], **o)
    assert NAMES[int(st[0])] == expected
    assert (int(st[0]), int(words[0])) == oracle.validate(build(), **o)


def test_reference_kats_host_mirror():
    msg = cp.Message.init(KATS[0][1]())
    assert msg.validate() == 3
    with pytest.raises(cp.TraversalLimitExceeded):
        msg.validate(traversal_limit_words=1, nesting_limit=64)
    with pytest.raises(cp.NestingLimitExceeded):
        msg.validate(nesting_limit=0)
    two = cp.Message.init(KATS[3][1]())
    two.validate(segment_count_limit=2)
    with pytest.raises(cp.SegmentCountLimitExceeded):
        two.validate(segment_count_limit=1)
    one = cp.Message.init(KATS[5][1]())
    assert one.validate(traversal_limit_words=1) == 1
    with pytest.raises(cp.TraversalLimitExceeded):
        one.validate(traversal_limit_words=0)
    three = cp.Message.init(KATS[7][1]())
    assert three.validate(nesting_limit=3) == 3
    with pytest.raises(cp.NestingLimitExceeded):
        three.validate(nesting_limit=2)


LIMITS = [
    dict(segment_count_limit=512, traversal_limit_words=8 * 1024 * 1024, nesting_limit=64),
    dict(segment_count_limit=512, traversal_limit_words=40, nesting_limit=64),
    dict(segment_count_limit=512, traversal_limit_words=8 * 1024 * 1024, nesting_limit=3),
    dict(segment_count_limit=2, traversal_limit_words=100, nesting_limit=5),
]


@pytest.mark.parametrize("k", range(len(LIMITS)))
def test_corpus_parity(k):
    msgs = msggen.corpus(200 + k, 6000)
    seen = check_against_oracle(msgs, LIMITS[k], pad_seed=k)
    assert len(seen) >= 5


def test_far_heavy_corpus_parity():
    rng = np.random.default_rng(91)
    msgs = []
    for _ in range(6000):
        m = msggen.random_message(rng, n_segments=int(rng.integers(2, 6)), far_rate=0.8, max_depth=8)
        msgs.append(msggen.mutate(rng, m) if rng.random() < 0.6 else m)
    seen = check_against_oracle(msgs, LIMITS[0], pad_seed=5)
    assert {0, CODES["InvalidFarPointer"], CODES["InvalidSegmentId"], CODES["OutOfBounds"]} <= seen


def test_reference_fuzz_shape_raw_and_packed():
    rng = np.random.default_rng(0xA7C41E59)
    raw = [rng.integers(0, 256, int(rng.integers(0, 160)), dtype=np.uint8).tobytes() for _ in range(4096)]
    unpacked = []
    for b in raw:
        st, u = oracle.unpack(b)
        if st == oracle.OK:
            unpacked.append(u)
    check_against_oracle(raw, LIMITS[0], pad_seed=7)
    check_against_oracle(unpacked, LIMITS[0], pad_seed=8)


def test_nesting_at_stack_depth():
    msgs = [msggen.deep_chain(d) for d in (1, 2, 63, 64, 65, 200)]
    st, words = run_batch(msgs, nesting_limit=64)
    exp = [oracle.validate(m, nesting_limit=64) for m in msgs]
    assert [(int(a), int(b)) for a, b in zip(st, words)] == exp
    assert exp[3] == (0, 64) and NAMES[exp[4][0]] == "NestingLimitExceeded"


def test_wide_and_long_lists():
    b = msggen.Builder(2)
    b.alloc(0, 1)
    n_ptr = 200_000
    lst = b.alloc(0, n_ptr)
    b.set(0, 0, msggen.list_ptr(lst - 1, 6, n_ptr))
    rng = np.random.default_rng(3)
    for i in rng.choice(n_ptr, 5000, replace=False):
        i = int(i)
        if rng.random() < 0.5:  # a 1-word struct in segment 1 through a single far pointer
            pad = b.alloc(1, 2)
            b.set(1, pad, msggen.struct_ptr(0, 1, 0))
            b.set(0, lst + i, msggen.far_ptr(False, pad, 1))
        else:  # a u64 list next to the pointer list
            at = b.alloc(0, 40)
            b.set(0, lst + i, msggen.list_ptr(at - (lst + i) - 1, 5, 40))
    m = b.framed()
    bad = bytearray(m)
    bad[-3] ^= 0x40
    msgs = [m, bytes(bad)]
    for opts in (LIMITS[0], dict(LIMITS[0], traversal_limit_words=n_ptr + 1000)):
        check_against_oracle(msgs, opts)


def test_empty_batch_and_argument_errors():
    d = torch.zeros(16, dtype=torch.uint8, device=DEV)
    z = torch.zeros(0, dtype=torch.int64, device=DEV)
    cp.validate_batch(d, z, z, torch.zeros(0, dtype=torch.int32, device=DEV))  # n = 0: no launch
    off = torch.zeros(1, dtype=torch.int64, device=DEV)
    ln = torch.full((1,), 16, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    with pytest.raises(cp.InvalidArgument):
        cp.validate_batch(d, off, ln, torch.zeros(0, dtype=torch.int32, device=DEV))


def test_words_optional():
    msgs = msggen.corpus(9, 500)
    st, _ = run_batch(msgs)
    d_st = torch.full((len(msgs),), -1, dtype=torch.int32, device=DEV)
    blob = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    offs = np.cumsum([0] + [len(m) for m in msgs[:-1]])
    cp.validate_batch(torch.from_numpy(blob.copy()).to(DEV), torch.tensor(offs, device=DEV),
                      torch.tensor([len(m) for m in msgs], device=DEV), d_st)
    assert np.array_equal(d_st.cpu().numpy(), st)


FIXTURES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")
PACKED_TWINS = (("packed", "binary"), ("segmented-packed", "segmented"),
                ("fixture_single_packed.bin", "fixture_single.bin"), ("fixture_far_packed.bin", "fixture_far.bin"))


def reference_messages():
    """The reference's framed messages (capnp testdata, interop fixtures) and the
    unpackPacked forms of their packed twins."""
    rd = lambda n: open(os.path.join(FIXTURES, n), "rb").read()
    msgs = {n: rd(n) for n in ("binary", "segmented", "fixture_single.bin", "fixture_far.bin")}
    for packed, _ in PACKED_TWINS:
        st, u = oracle.unpack(rd(packed))
        assert st == oracle.OK
        msgs[packed + " (unpacked)"] = u
    return msgs


def test_reference_messages_default_limits():
    msgs = reference_messages()
    for pad in (None, 3):
        check_against_oracle(list(msgs.values()), LIMITS[0], pad_seed=pad)
    st, words = run_batch(list(msgs.values()))
    assert all(int(x) == 0 for x in st)  # the reference's own messages are valid
    assert int(words[0]) == 348 and int(words[2]) == 34 and int(words[3]) == 34


def test_reference_messages_tight_limits():
    for name, m in reference_messages().items():
        _, w = oracle.validate(m)
        nseg = int.from_bytes(m[:4], "little") + 1
        sets = [dict(LIMITS[0], traversal_limit_words=t) for t in {max(w - 1, 0), w, w + 1, 1, 0}]
        sets += [dict(LIMITS[0], nesting_limit=k) for k in (0, 1, 2, 3, 4, 5, 6, 100)]
        sets += [dict(LIMITS[0], segment_count_limit=k) for k in {nseg - 1, nseg, 1}]
        for opts in sets:
            check_against_oracle([m], opts)


@pytest.mark.parametrize("nesting", [65, 100, 200, 1000, 0xFFFFFFFF])
def test_nesting_above_stack_depth(nesting):
    chains = [msggen.deep_chain(d) for d in (1, 63, 64, 65, 100, 199, 200, 201, 300)]
    seen = check_against_oracle(chains, dict(LIMITS[0], nesting_limit=nesting))
    st, words = run_batch([msggen.deep_chain(200)], nesting_limit=200)
    assert (int(st[0]), int(words[0])) == (0, 200)  # verdict ask: a depth-200 chain at limit 200
    assert (CODES["NestingLimitExceeded"] in seen) == (nesting < 300)


@pytest.mark.parametrize("nesting", [70, 150, 400])
def test_deep_mixed_spines_among_shallow_messages(nesting):
    """Deep spines of every pointer kind (near and far links) interleaved with a damaged
    shallow corpus: only the deep ones take the deep pass, every status and word count
    equals the oracle's, including errors raised inside the deep part."""
    rng = np.random.default_rng(nesting)
    shallow = msggen.corpus(40 + nesting, 3000)
    deep = [msggen.deep_mixed(rng, int(rng.integers(30, 260))) for _ in range(120)]
    deep += [msggen.mutate(rng, msggen.deep_mixed(rng, int(rng.integers(60, 200)))) for _ in range(120)]
    msgs = shallow[:]
    for i, m in enumerate(deep):
        msgs.insert(int(rng.integers(0, len(msgs) + 1)), m)
    for opts in (dict(LIMITS[0], nesting_limit=nesting), dict(LIMITS[0], nesting_limit=nesting, traversal_limit_words=300)):
        check_against_oracle(msgs, opts, pad_seed=nesting)


def test_deep_limit_equal_to_traversal():
    """The deep pass's frame stacks are sized by min(nesting, traversal limit)."""
    msgs = [msggen.deep_chain(d) for d in (100, 150, 151, 400)]
    for trav in (1, 150, 151, 1 << 40):
        check_against_oracle(msgs, dict(LIMITS[0], nesting_limit=1 << 20, traversal_limit_words=trav))
