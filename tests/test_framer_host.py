"""Host logic of PackedConnections.handle_read, on CPU: the native entry point
capnp_packed_frame_connections is replaced by a stand-in that follows its header
contract (include/capnp_packed.h) with the oracle's Reader.readPackedMessage
(reader.zig:84-156), one unit per live connection per round. What is tested is the
Python side: the input layout, frames grouped per connection in pop order, the bytes
left in each framer, errors closing a connection (connection.zig:175-184) with its
earlier frames in frames_before_error, and the OUT_OF_SPACE retry of the whole call.
The device path itself is tested in test_gpu_framer.py."""
import ctypes

import numpy as np
import pytest

import capnp_packed as cp
import oracle
import pyref

ORACLE_TO_ABI = {0: cp.OK, -1: cp.END_OF_STREAM, -2: cp.INVALID_SEGMENT_COUNT,
                 -3: cp.SEGMENT_COUNT_LIMIT_EXCEEDED, -6: cp.MESSAGE_TOO_LARGE, -7: cp.INVALID_PACKED_MESSAGE}


def _arr(ptr, n, ctype):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctype)), shape=(max(n, 1),))


class FakeFramer:
    """capnp_packed_frame_connections restated on the oracle reader (test stand-in)."""

    def __init__(self, fail_first=0):
        self.calls = 0
        self.fail_first = fail_first  # the first calls report OUT_OF_SPACE (frames too small)

    def __call__(self, inp, in_bytes, in_off, in_len, n, slot_guess, frames, frames_cap, f_off, f_len, f_conn,
                 max_frames, consumed, status, n_frames):
        self.calls += 1
        if self.calls <= self.fail_first:
            return cp.OUT_OF_SPACE
        data = bytes(_arr(inp, in_bytes, ctypes.c_uint8)[:in_bytes])
        off, ln = _arr(in_off, n, ctypes.c_uint64), _arr(in_len, n, ctypes.c_uint64)
        guess = _arr(slot_guess, n, ctypes.c_uint64)
        fr = _arr(frames, frames_cap, ctypes.c_uint8)
        fo, fl = _arr(f_off, max_frames, ctypes.c_uint64), _arr(f_len, max_frames, ctypes.c_uint64)
        fc = _arr(f_conn, max_frames, ctypes.c_uint32)
        cons, st = _arr(consumed, n, ctypes.c_uint64), _arr(status, n, ctypes.c_int32)
        used = [0] * n
        live = [int(ln[c]) > 0 for c in range(n)]
        for c in range(n):
            st[c] = cp.END_OF_STREAM
        cur = nf = 0
        while True:
            idx = [c for c in range(n) if live[c] and used[c] < int(ln[c])]
            if not idx:
                break
            for c in idx:  # one round: the next message of each live connection
                buf = data[int(off[c]) + used[c]:int(off[c]) + int(ln[c])]
                rc, framed, u = oracle.read_packed_message(buf, cap=1 << 22)
                rc = ORACLE_TO_ABI[rc]
                if rc == cp.OK:
                    if cur + len(framed) > frames_cap or nf >= max_frames:
                        return cp.OUT_OF_SPACE
                    fr[cur:cur + len(framed)] = np.frombuffer(framed, dtype=np.uint8)
                    fo[nf], fl[nf], fc[nf] = cur, len(framed), c
                    nf += 1
                    cur += (len(framed) + 7) // 8 * 8
                    used[c] += u
                    guess[c] = max(8, len(framed))
                else:
                    live[c] = False
                    st[c] = rc
        for c in range(n):
            cons[c] = used[c]
        n_frames._obj.value = nf
        return cp.OK


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


@pytest.mark.parametrize("fail_first", [0, 2])
def test_handle_read_host_logic(monkeypatch, fail_first):
    fake = FakeFramer(fail_first)
    monkeypatch.setattr(cp.lib(), "capnp_packed_frame_connections", fake)
    rng = np.random.default_rng(0x5EED + fail_first)
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
            assert c not in errors and bytes(conns.framers[c].buffer) == (rest if rc else b"")
        else:
            assert errors[c].status == rc and conns.closed[c] and conns.framers[c].buffered_bytes() == 0
    assert fake.calls >= 3 + fail_first
