"""Host-side framing mirror (MessageBuilder.toBytes / Message.init), CPU-only.
message.zig:2123-2170 (toBytes) and :341-394 (Message.init)."""
import os

import pytest

import capnp_packed as cp
import oracle
import pyref

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")


def fx(name):
    return open(os.path.join(FIX, name), "rb").read()


@pytest.mark.parametrize("name", ["binary", "segmented", "fixture_single.bin", "fixture_far.bin"])
def test_message_init_matches_oracle_on_fixtures(name):
    data = fx(name)
    rc, segs = oracle.message_init(data)
    assert rc == 0
    msg = cp.Message.init(data)
    assert [(s.obj is not None, len(s)) for s in msg.segments] == [(True, ln) for _, ln in segs]
    assert [bytes(s) for s in msg.segments] == [data[o:o + ln] for o, ln in segs]


def test_fixture_segment_counts():
    assert len(cp.Message.init(fx("binary")).segments) == 1
    assert len(cp.Message.init(fx("fixture_far.bin")).segments) == 4
    assert len(cp.Message.init(fx("segmented")).segments) > 100


def test_builder_to_bytes_roundtrip():
    b = cp.MessageBuilder()
    b.create_segment(bytes(range(16)))
    b.create_segment(bytes(8))
    framed = b.to_bytes()
    assert framed == pyref.frame([bytes(range(16)), bytes(8)])
    msg = cp.Message.init(framed)
    assert [bytes(s) for s in msg.segments] == [bytes(range(16)), bytes(8)]


def test_empty_builder_has_one_segment():
    assert cp.MessageBuilder().to_bytes() == pyref.frame([b""])


@pytest.mark.parametrize("data,exc", [
    (b"", cp.EndOfStream),
    (b"\xff\xff\xff\xff", cp.InvalidSegmentCount),
    ((512).to_bytes(4, "little") + bytes(4), cp.SegmentCountLimitExceeded),
    ((1).to_bytes(4, "little") + bytes(4), cp.TruncatedMessage),
    (bytes(4) + (2).to_bytes(4, "little") + bytes(8), cp.TruncatedMessage),
])
def test_message_init_errors(data, exc):
    with pytest.raises(exc):
        cp.Message.init(data)


def test_validate_of_message_without_segments_is_empty_message():
    # message.zig:700: validate on a message with no segments (e.g. after deinit) raises
    # EmptyMessage before any device work
    m = cp.Message.init(open(os.path.join(FIX, "fixture_single.bin"), "rb").read())
    m.deinit()
    with pytest.raises(cp.EmptyMessage):
        m.validate()
    with pytest.raises(cp.EmptyMessage):
        cp.Message([], None).validate()
