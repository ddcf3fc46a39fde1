"""Message.validate oracle (oracle_validate, message.zig:699-969) pinned on CPU:

- the reference's own known-answer tests (tests/serialization/message_test.zig:184-260),
  on the C oracle and on the pure-Python restatement (tests/pyref.py);
- the two restatements against each other on random message trees with every pointer
  encoding, most of them damaged (tests/msggen.py), under varied limits: same first
  error, same traversal words;
- the reference's malformed-buffer fuzz shape (message_test.zig:1057-1093: 1024 random
  buffers shorter than 160 bytes, raw and through unpackPacked); the generator is
  numpy's, not Zig's DefaultPrng, so the buffers differ from the reference's but have
  its distribution: agreement, no crash.
"""
import numpy as np
import pytest

import msggen
import oracle
import pyref
from validate_cases import CODES, KATS, NAMES, kat_options, limits_for


def py_status(data, **opts):
    try:
        return 0, pyref.validate(data, **opts)
    except pyref.ValidateError as e:
        return CODES[e.args[0]], 0


@pytest.mark.parametrize("name,build,opts,expected", KATS, ids=[k[0] for k in KATS])
def test_reference_kats(name, build, opts, expected):
    o = kat_options(opts)
    st, _ = oracle.validate(build(), **o)
    assert NAMES[st] == expected
    pst, _ = py_status(build(), **o)
    assert NAMES[pst] == expected


def test_kat_traversal_words():
    # struct (1, 1) + "hello": 2 struct words + 1 text word; the others as built
    assert oracle.validate(KATS[0][1]())[1] == 3
    assert oracle.validate(KATS[5][1](), traversal_limit_words=1) == (0, 1)
    assert oracle.validate(KATS[7][1](), nesting_limit=3) == (0, 3)


def test_deep_chain_nesting_boundary():
    for depth in (1, 2, 31, 64):
        m = msggen.deep_chain(depth)
        assert oracle.validate(m, nesting_limit=depth) == (0, depth)
        assert oracle.validate(m, nesting_limit=depth - 1)[0] == CODES["NestingLimitExceeded"]
        assert py_status(m, nesting_limit=depth) == (0, depth)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_matches_python_restatement(seed):
    rng = np.random.default_rng(1000 + seed)
    msgs = msggen.corpus(seed, 700)
    seen = set()
    for i, m in enumerate(msgs):
        o = limits_for(rng, i)
        got = oracle.validate(m, **o)
        exp = py_status(m, **o)
        assert got == exp, f"message {i}: oracle {got} python {exp} ({o})"
        seen.add(got[0])
    # the corpus reaches the walk's error paths, not only the happy path
    for name in ("OutOfBounds", "TraversalLimitExceeded", "NestingLimitExceeded", "InvalidPointer",
                 "InvalidSegmentId", "SegmentCountLimitExceeded"):
        assert CODES[name] in seen, f"{name} never reached"
    assert 0 in seen


def test_far_and_composite_error_paths_reached():
    rng = np.random.default_rng(77)
    seen = set()
    for i in range(3000):
        m = msggen.mutate(rng, msggen.random_message(rng, n_segments=3, far_rate=0.8))
        st, _ = oracle.validate(m)
        assert (st, _) == py_status(m)
        seen.add(st)
    assert {CODES["InvalidFarPointer"], CODES["InvalidInlineCompositePointer"]} <= seen


def test_reference_fuzz_shape_raw_and_packed():
    rng = np.random.default_rng(0x3E227AB4)
    for _ in range(1024):
        b = rng.integers(0, 256, int(rng.integers(0, 160)), dtype=np.uint8).tobytes()
        assert oracle.validate(b) == py_status(b)
        st, unpacked = oracle.unpack(b)
        if st == oracle.OK:
            assert oracle.validate(unpacked) == py_status(unpacked)


def test_valid_trees_validate():
    rng = np.random.default_rng(5)
    for _ in range(300):
        m = msggen.random_message(rng)
        st, words = oracle.validate(m)
        assert st == 0 and words <= len(m) // 8


def test_generator_read_count_matches_walk():
    # msggen's per-tree count of the words the walk reads (bench.py's algorithmic bytes
    # for the validate leg) equals the restatement's own count of word reads
    class Counting(pyref._Validator):
        n = 0

        def word(self, seg, pos):
            Counting.n += 1
            return super().word(seg, pos)

    rng = np.random.default_rng(11)
    for _ in range(200):
        t = msggen.RandomTree(rng)
        segs = pyref.message_segments(t.framed())
        Counting.n = 0
        v = Counting(segs, 1 << 40)
        v.pointer(0, 0, v.word(0, 0), 64)
        assert Counting.n == t.reads


def test_reference_messages_validate_on_the_oracle():
    """The reference's real messages (capnp testdata, interop fixtures) and the unpacked
    forms of their packed twins: valid under the default limits, the twins identical to
    the framed files, and the limit edges the GPU tests compare at behave as expected."""
    import os
    fx = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")
    rd = lambda n: open(os.path.join(fx, n), "rb").read()
    expect = {"binary": 348, "segmented": 0, "fixture_single.bin": 34, "fixture_far.bin": 34}
    for name, words in expect.items():
        assert oracle.validate(rd(name)) == (0, words)
    for packed, twin in (("packed", "binary"), ("segmented-packed", "segmented"),
                         ("fixture_single_packed.bin", "fixture_single.bin"),
                         ("fixture_far_packed.bin", "fixture_far.bin")):
        st, u = oracle.unpack(rd(packed))
        assert st == oracle.OK and u == rd(twin)
    m = rd("binary")
    assert oracle.validate(m, traversal_limit_words=347)[0] == CODES["TraversalLimitExceeded"]
    assert oracle.validate(m, nesting_limit=4)[0] == CODES["NestingLimitExceeded"]
    assert oracle.validate(m, nesting_limit=5) == (0, 348)
    # segmented's root is a double far whose pad holds a struct tag: validateFarPointer
    # reads it as an inline-composite tag of count 0 (:765-767) and stops
    assert oracle.validate(rd("segmented"), segment_count_limit=124)[0] == CODES["SegmentCountLimitExceeded"]


def test_deep_nesting_on_the_oracle():
    import numpy as np
    for d in (64, 65, 200):
        assert oracle.validate(msggen.deep_chain(d), nesting_limit=d) == (0, d)
        assert oracle.validate(msggen.deep_chain(d), nesting_limit=d - 1)[0] == CODES["NestingLimitExceeded"]
    rng = np.random.default_rng(5)
    m = msggen.deep_mixed(rng, 100)
    st, w = oracle.validate(m, nesting_limit=1000)
    assert st == 0 and w > 100
