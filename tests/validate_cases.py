"""Shared Message.validate test cases (test-only): the reference's known-answer tests
(tests/serialization/message_test.zig:184-260) rebuilt with tests/msggen.py, and the
status-code <-> reference-error-name map of include/capnp_packed.h."""
import msggen
from msggen import Builder, list_ptr, struct_ptr

NAMES = {
    0: None,
    8: "EndOfStream",
    9: "InvalidSegmentCount",
    10: "SegmentCountLimitExceeded",
    13: "TruncatedMessage",
    14: "EmptyMessage",
    15: "NestingLimitExceeded",
    16: "InvalidSegmentId",
    17: "InvalidPointer",
    18: "OutOfBounds",
    19: "TraversalLimitExceeded",
    20: "InvalidFarPointer",
    21: "InvalidInlineCompositePointer",
    22: "ListTooLarge",
}
CODES = {v: k for k, v in NAMES.items()}


def msg_struct_with_text() -> bytes:
    """message_test.zig:185-192: allocateStruct(1, 1), writeU64(0, 42), writeText(0, "hello")."""
    b = Builder(1)
    b.alloc(0, 1)
    s = b.alloc(0, 2)
    b.set(0, 0, struct_ptr(s - 1, 1, 1))
    b.set(0, s, 42)
    t = b.alloc(0, 1)
    b.set(0, s + 1, list_ptr(t - (s + 1) - 1, 2, 6))  # "hello\0": byte list of 6
    b.set(0, t, int.from_bytes(b"hello\0\0\0", "little"))
    return b.framed()


def msg_two_segments() -> bytes:
    """message_test.zig:210-216: allocateStruct(0, 0) then createSegment()."""
    b = Builder(2)
    b.alloc(0, 1)
    b.set(0, 0, struct_ptr(0, 0, 0))
    return b.framed()


def msg_struct_1_0() -> bytes:
    """message_test.zig:227-233: allocateStruct(1, 0), writeU64(0, 123)."""
    b = Builder(1)
    b.alloc(0, 1)
    s = b.alloc(0, 1)
    b.set(0, 0, struct_ptr(s - 1, 1, 0))
    b.set(0, s, 123)
    return b.framed()


def msg_three_levels() -> bytes:
    """message_test.zig:244-252: root (0, 1) -> child (0, 1) -> grandchild (1, 0) = 99."""
    b = Builder(1)
    b.alloc(0, 1)
    r = b.alloc(0, 1)
    b.set(0, 0, struct_ptr(r - 1, 0, 1))
    c = b.alloc(0, 1)
    b.set(0, r, struct_ptr(c - r - 1, 0, 1))
    g = b.alloc(0, 1)
    b.set(0, c, struct_ptr(g - c - 1, 1, 0))
    b.set(0, g, 99)
    return b.framed()


DEFAULTS = dict(segment_count_limit=512, traversal_limit_words=8 * 1024 * 1024, nesting_limit=64)

# (test name at message_test.zig:line, message, options, expected error name or None)
KATS = [
    ("validate traversal and nesting limits :198", msg_struct_with_text, {}, None),
    ("validate traversal and nesting limits :199", msg_struct_with_text,
     dict(traversal_limit_words=1, nesting_limit=64), "TraversalLimitExceeded"),
    ("validate traversal and nesting limits :200", msg_struct_with_text, dict(nesting_limit=0),
     "NestingLimitExceeded"),
    ("validate enforces segment count limit option :222", msg_two_segments, dict(segment_count_limit=2), None),
    ("validate enforces segment count limit option :223", msg_two_segments, dict(segment_count_limit=1),
     "SegmentCountLimitExceeded"),
    ("traversal limit boundary conditions :239", msg_struct_1_0, dict(traversal_limit_words=1), None),
    ("traversal limit boundary conditions :240", msg_struct_1_0, dict(traversal_limit_words=0),
     "TraversalLimitExceeded"),
    ("nesting limit boundary conditions :258", msg_three_levels, dict(nesting_limit=3), None),
    ("nesting limit boundary conditions :259", msg_three_levels, dict(nesting_limit=2), "NestingLimitExceeded"),
]


def kat_options(opts):
    o = dict(DEFAULTS)
    o.update(opts)
    return o


def limits_for(rng, i):
    """Per-message validation options for the parity corpora: mostly the defaults,
    some tight traversal / nesting / segment limits so their boundaries are crossed."""
    r = i % 5
    if r == 0:
        return dict(DEFAULTS)
    if r == 1:
        return dict(DEFAULTS, traversal_limit_words=int(rng.integers(0, 64)))
    if r == 2:
        return dict(DEFAULTS, nesting_limit=int(rng.integers(0, 8)))
    if r == 3:
        return dict(DEFAULTS, segment_count_limit=int(rng.integers(1, 5)))
    return dict(segment_count_limit=int(rng.integers(1, 6)), traversal_limit_words=int(rng.integers(0, 200)),
                nesting_limit=int(rng.integers(0, 65)))


__all__ = ["NAMES", "CODES", "KATS", "kat_options", "limits_for", "msggen"]
