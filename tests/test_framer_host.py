"""Host logic of PackedConnections.handle_read and PackedFramer, on CPU: the native
session (FramerSession over capnp_packed_framer_*) is replaced by a stand-in that follows
its header contract (include/capnp_packed.h) with the oracle's Reader.readPackedMessage
(reader.zig:84-156). What is tested is the Python side: frames grouped per connection in pop
order, errors closing a connection (connection.zig:175-184) with its earlier frames in
frames_before_error, the bytes each framer keeps, and PackedFramer's pop / error / reset
order. The device path itself is tested in test_gpu_framer.py."""
import numpy as np
import pytest

import capnp_packed as cp
import oracle
import pyref

ORACLE_TO_ABI = {0: cp.OK, -1: cp.END_OF_STREAM, -2: cp.INVALID_SEGMENT_COUNT,
                 -3: cp.SEGMENT_COUNT_LIMIT_EXCEEDED, -6: cp.MESSAGE_TOO_LARGE, -7: cp.INVALID_PACKED_MESSAGE}


class FakeSession:
    """capnp_packed_framer_* restated on the oracle reader (test stand-in)."""

    def __init__(self, n_conns):
        self.n = n_conns
        self.buf = [b""] * n_conns
        self.calls = 0

    def read(self, reads):
        self.calls += 1
        for c, d in reads.items():
            self.buf[c] += bytes(d)
        frames, status = {}, np.full(self.n, cp.END_OF_STREAM, dtype=np.int32)
        for c in range(self.n):
            while self.buf[c]:
                rc, framed, used = oracle.read_packed_message(self.buf[c], cap=1 << 22)
                rc = ORACLE_TO_ABI[rc]
                if rc == cp.END_OF_STREAM:
                    break
                if rc != cp.OK:
                    status[c] = rc
                    self.buf[c] = b""  # the session drops a failed connection's bytes
                    break
                frames.setdefault(c, []).append(memoryview(framed))
                self.buf[c] = self.buf[c][used:]
        return frames, status

    def buffered(self, c):
        return len(self.buf[c])

    def reset(self, c):
        self.buf[c] = b""


def make_stream(rng, n_msgs):
    packed = []
    for _ in range(n_msgs):
        segs = []
        for _ in range(int(rng.integers(1, 4))):
            m = 8 * int(rng.integers(0, 64))
            b = rng.integers(0, 256, m).astype(np.uint8)
            b[rng.random(m) < 0.5] = 0
            segs.append(b.tobytes())
        st, p = oracle.pack(pyref.frame(segs))
        assert st == oracle.OK
        packed.append(p)
    return packed


def oracle_frames(data: bytes):
    frames = []
    while data:
        rc, framed, used = oracle.read_packed_message(data, cap=1 << 22)
        if rc != 0:
            return frames, data, ORACLE_TO_ABI[rc]
        frames.append(framed)
        data = data[used:]
    return frames, data, cp.OK


def test_handle_read_host_logic(monkeypatch):
    monkeypatch.setattr(cp, "FramerSession", FakeSession)
    rng = np.random.default_rng(0x5EED)
    n_conns = 23
    bad = bytes([0x03, 0x57, 0x02])  # segment count 600 > 512
    streams, expect = [], []
    for c in range(n_conns):
        packed = make_stream(rng, int(rng.integers(0, 6)))
        data = b"".join(packed)
        if c % 7 == 3 and packed:  # one good message, then a bad header
            data = packed[0] + bad + b"".join(packed[1:])
        streams.append(data)
        expect.append(oracle_frames(data))
    conns = cp.PackedConnections(n_conns, device="cpu")
    reads = []
    for s in streams:  # 3 socket reads per connection, cut anywhere
        cut = sorted(rng.integers(0, len(s) + 1, 2).tolist())
        reads.append([s[:cut[0]], s[cut[0]:cut[1]], s[cut[1]:]])
    delivered = [[] for _ in range(n_conns)]
    errors = {}
    for r in range(3):
        res = conns.handle_read({c: reads[c][r] for c in range(n_conns)})
        for c, v in res.items():
            if isinstance(v, cp.PackedError):
                errors[c] = v
                delivered[c] += conns.frames_before_error.get(c, [])
            else:
                delivered[c] += [bytes(f) for f in v]
    for c in range(n_conns):
        frames, rest, rc = expect[c]
        assert [bytes(f) for f in delivered[c]] == frames, f"connection {c}"
        if rc in (cp.OK, cp.END_OF_STREAM):
            assert c not in errors and conns.framers[c].buffered_bytes() == (len(rest) if rc else 0)
        else:
            assert errors[c].status == rc and conns.closed[c] and conns.framers[c].buffered_bytes() == 0
    assert conns.session.calls == 3


def test_packed_framer_host_logic(monkeypatch):
    """PackedFramer over the session: frames in push order, None while a message is
    incomplete (bytes kept), the reader's error after the frames before it, reset."""
    monkeypatch.setattr(cp, "FramerSession", FakeSession)
    rng = np.random.default_rng(0xF00D)
    packed = make_stream(rng, 5)
    msgs = [oracle.read_packed_message(p, cap=1 << 22)[1] for p in packed]
    f = cp.PackedFramer()
    stream = b"".join(packed)
    got = []
    for i in range(0, len(stream), 37):
        f.push(stream[i:i + 37])
        while (fr := f.pop_frame()) is not None:
            got.append(fr)
    assert got == msgs and f.buffered_bytes() == 0
    f.push(packed[0][:-1])
    assert f.pop_frame() is None and f.buffered_bytes() == len(packed[0]) - 1
    f.push(packed[0][-1:] + packed[1] + bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF]))
    assert f.pop_frame() == msgs[0] and f.pop_frame() == msgs[1]
    with pytest.raises(cp.PackedError) as e:
        f.pop_frame()
    assert e.value.status == cp.INVALID_SEGMENT_COUNT
    f.reset()
    assert f.buffered_bytes() == 0 and f.pop_frame() is None


def test_framer_session_groups_frames_per_connection():
    """FramerSession.read's grouping of the native calls' frame tables (no device): frames of a
    connection in order across calls, whether a call's table is already grouped by connection
    (one walk pass) or interleaved (several passes), as read-only views of the call's buffer."""
    sess = object.__new__(cp.FramerSession)
    sess.n, sess.handle = 4, None
    buf1 = np.frombuffer(b"".join(bytes([i]) * 8 for i in range(6)), dtype=np.uint8).copy()
    buf2 = np.frombuffer(b"".join(bytes([100 + i]) * 8 for i in range(5)), dtype=np.uint8).copy()
    u64 = lambda xs: np.array(xs, dtype=np.uint64)  # noqa: E731
    parts = [  # call 1: grouped (connections 0, 0, 1, 3, 3, 3); call 2: interleaved passes
        (buf1, u64([0, 8, 16, 24, 32, 40]), u64([8] * 6), np.array([0, 0, 1, 3, 3, 3], dtype=np.uint32)),
        (buf2, u64([0, 8, 16, 24, 32]), u64([8] * 5), np.array([1, 3, 0, 1, 3], dtype=np.uint32)),
    ]
    status = np.full(4, cp.END_OF_STREAM, dtype=np.int32)
    sess.readv_raw = lambda reads: (parts, status)
    frames, st = sess.read({0: b"x"})
    got = {c: [bytes(v) for v in fr] for c, fr in frames.items()}
    assert got == {0: [bytes([0]) * 8, bytes([1]) * 8, bytes([102]) * 8],
                   1: [bytes([2]) * 8, bytes([100]) * 8, bytes([103]) * 8],
                   3: [bytes([3]) * 8, bytes([4]) * 8, bytes([5]) * 8, bytes([101]) * 8, bytes([104]) * 8]}
    assert all(v.readonly for fr in frames.values() for v in fr) and (st == cp.END_OF_STREAM).all()
