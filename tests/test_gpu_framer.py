"""framing packed byte streams as they come off a socket.
`PackedFramer` mirrors the RPC Framer (src/rpc/level0/framing.zig:4-90: push /
bufferedBytes / reset / popFrame) for a packed stream. `PackedConnections` runs
Connection.handleRead (src/rpc/level2/connection.zig:153-203) for many connections in
one device batch per round.

The expected frames are the framed messages the streams were built from. Every popped
frame and error is also checked against the oracle's restatement of
Reader.readPackedMessage (reader.zig:84-156), applied to the same buffered bytes.
"""
import numpy as np
import pytest

import capnp_packed as cp
import oracle
import pyref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
# oracle_read_packed_message's codes -> the C-ABI statuses (as in test_gpu_read_message.py)
ORACLE_TO_ABI = {0: cp.OK, -1: cp.END_OF_STREAM, -2: cp.INVALID_SEGMENT_COUNT,
                 -3: cp.SEGMENT_COUNT_LIMIT_EXCEEDED, -6: cp.MESSAGE_TOO_LARGE, -7: cp.INVALID_PACKED_MESSAGE}


def random_message(rng):
    segs = []
    for _ in range(int(rng.integers(1, 5))):
        n = 8 * int(rng.integers(0, 160))
        b = rng.integers(0, 256, n).astype(np.uint8)
        b[rng.random(n) < rng.choice([0.1, 0.5, 0.9])] = 0
        segs.append(b.tobytes())
    return pyref.frame(segs)


def make_stream(rng, n_msgs):
    msgs = [random_message(rng) for _ in range(n_msgs)]
    packed = []
    for f in msgs:
        st, p = oracle.pack(f)
        assert st == oracle.OK
        packed.append(p)
    return msgs, packed


def oracle_frames(data: bytes):
    """Pop frames from `data` with the oracle reader until it stops: (frames, rest, code)."""
    frames = []
    while data:
        rc, framed, used = oracle.read_packed_message(data, cap=1 << 22)
        if rc == -8:  # the oracle's output buffer: up to the 8 Mi-word limit (framing.zig:5)
            rc, framed, used = oracle.read_packed_message(data, cap=8 * (8 * 1024 * 1024 + 520))
        if rc != 0:
            return frames, data, ORACLE_TO_ABI[rc]
        frames.append(framed)
        data = data[used:]
    return frames, data, cp.OK


def chunks(rng, data: bytes, k: int):
    cut = sorted(rng.integers(0, len(data) + 1, k - 1).tolist()) if len(data) else [0] * (k - 1)
    edges = [0] + cut + [len(data)]
    return [data[edges[i]:edges[i + 1]] for i in range(k)]


def test_packed_framer_socket_reads():
    rng = np.random.default_rng(0xF4A3)
    msgs, packed = make_stream(rng, 24)
    stream = b"".join(packed)
    f = cp.PackedFramer()
    got = []
    for piece in chunks(rng, stream, 40):  # socket reads of arbitrary sizes
        f.push(piece)
        while True:
            fr = f.pop_frame()
            if fr is None:
                break
            got.append(fr)
    assert got == msgs and f.buffered_bytes() == 0
    # a read that ends inside a message keeps the bytes (popFrame's null)
    f.push(packed[0][:-1])
    assert f.pop_frame() is None and f.buffered_bytes() == len(packed[0]) - 1
    f.push(packed[0][-1:])
    assert f.pop_frame() == msgs[0]


def test_packed_framer_error_then_reset():
    rng = np.random.default_rng(7)
    msgs, packed = make_stream(rng, 2)
    bad = bytes([0x0F, 0xFF, 0xFF, 0xFF, 0xFF])  # segment count - 1 = 0xFFFFFFFF
    rc, _, _ = oracle.read_packed_message(bad + packed[1], cap=1 << 20)
    rc = ORACLE_TO_ABI[rc]
    assert rc == cp.INVALID_SEGMENT_COUNT
    f = cp.PackedFramer()
    f.push(packed[0] + bad + packed[1])
    assert f.pop_frame() == msgs[0]
    with pytest.raises(cp.PackedError) as e:
        f.pop_frame()
    assert e.value.status == rc
    f.reset()  # Connection.handleRead resets the framer after a framing error
    assert f.buffered_bytes() == 0 and f.pop_frame() is None


@pytest.mark.parametrize("n_conns", [1, 48])
def test_packed_connections_batched(n_conns):
    rng = np.random.default_rng(0xC0 + n_conns)
    bad = bytes([0x03, 0x57, 0x02])  # segment count 600 > 512
    streams, expect = [], []
    for c in range(n_conns):
        msgs, packed = make_stream(rng, int(rng.integers(0, 7)))
        data = b"".join(packed)
        if c % 11 == 5 and msgs:  # a corrupt connection: one good message, then garbage
            data = packed[0] + bad + b"".join(packed[1:])
        streams.append(data)
        expect.append(oracle_frames(data))
    conns = cp.PackedConnections(n_conns)
    reads = [chunks(rng, s, 4) for s in streams]
    delivered = [[] for _ in range(n_conns)]
    errors = {}
    for r in range(4):
        res = conns.handle_read({c: reads[c][r] for c in range(n_conns)})
        for c, v in res.items():
            if isinstance(v, cp.PackedError):
                errors[c] = v
                delivered[c] += conns.frames_before_error.get(c, [])
            else:
                delivered[c] += v
    for c in range(n_conns):
        frames, rest, rc = expect[c]
        assert delivered[c] == frames, f"connection {c}"
        if rc in (cp.OK, cp.END_OF_STREAM):
            assert c not in errors and conns.framers[c].buffered_bytes() == (len(rest) if rc else 0)
        else:
            assert errors[c].status == rc and conns.closed[c] and conns.framers[c].buffered_bytes() == 0


def _zero_heavy_message(words):
    """A 1-segment framed message of `words` zero words: 2 packed bytes per 256 words, so its
    framed length is far beyond any slot guessed from the packed size (the OUT_OF_SPACE
    round of capnp_packed_frame_connections)."""
    return pyref.frame([bytes(8 * words)])


def test_frame_connections_slot_growth_and_small_buffers():
    """capnp_packed_frame_connections through the C-ABI: frames of zero-run messages whose
    framed length is ~100x their packed bytes (each connection's slot grows across
    OUT_OF_SPACE rounds), empty connections beside them, a truncated last message, and a
    frame buffer / frame table too small (OUT_OF_SPACE for the call, then a retry)."""
    import ctypes
    rng = np.random.default_rng(0xF8)
    conns = []
    for c in range(40):
        msgs = []
        for _ in range(int(rng.integers(0, 4))):
            if rng.random() < 0.5:
                msgs.append(_zero_heavy_message(int(rng.integers(300, 20000))))
            else:
                msgs.append(random_message(rng))
        data = b"".join(oracle.pack(m)[1] for m in msgs)
        if c % 9 == 4 and data:
            data = data[:-1]  # the last message is cut short: END_OF_STREAM, its bytes kept
        conns.append(data)
    expect = [oracle_frames(d) for d in conns]
    lens = np.array([len(d) for d in conns], dtype=np.uint64)
    base = np.zeros(len(conns), dtype=np.uint64)
    base[1:] = np.cumsum(lens)[:-1]
    host = np.frombuffer(b"".join(conns) or b"\0", dtype=np.uint8)
    total = int(lens.sum())

    def call(frames_cap, max_frames):
        g = np.full(len(conns), 64, dtype=np.uint64)  # small guesses: every big frame grows its slot
        fr = np.zeros(max(frames_cap, 1), dtype=np.uint8)
        fo = np.zeros(max(max_frames, 1), dtype=np.uint64)
        fl = np.zeros(max(max_frames, 1), dtype=np.uint64)
        fc = np.zeros(max(max_frames, 1), dtype=np.uint32)
        cons = np.zeros(len(conns), dtype=np.uint64)
        st = np.zeros(len(conns), dtype=np.int32)
        nf = ctypes.c_uint32(0)
        rc = cp.lib().capnp_packed_frame_connections(
            host.ctypes.data, total, base.ctypes.data, lens.ctypes.data, len(conns), g.ctypes.data, fr.ctypes.data,
            frames_cap, fo.ctypes.data, fl.ctypes.data, fc.ctypes.data, max_frames, cons.ctypes.data,
            st.ctypes.data, ctypes.byref(nf))
        return rc, fr, fo, fl, fc, cons, st, nf.value

    assert call(64, 1024)[0] == cp.OUT_OF_SPACE   # frames do not fit
    assert call(1 << 26, 1)[0] == cp.OUT_OF_SPACE  # frame table too small
    rc, fr, fo, fl, fc, cons, st, n = call(1 << 26, 1024)
    assert rc == cp.OK
    got = [[] for _ in conns]
    for i in range(n):
        got[int(fc[i])].append(fr[int(fo[i]):int(fo[i]) + int(fl[i])].tobytes())
    for c, (frames, rest, code) in enumerate(expect):
        assert got[c] == frames, f"connection {c}"
        assert int(cons[c]) == len(conns[c]) - len(rest)
        assert int(st[c]) == (cp.END_OF_STREAM if code in (cp.OK, cp.END_OF_STREAM) else code)


def _frame_connections(streams, frames):
    """capnp_packed_frame_connections through the C-ABI with the caller's `frames` buffer."""
    import ctypes
    k = len(streams)
    lens = np.array([len(s) for s in streams], dtype=np.uint64)
    base = np.zeros(k, dtype=np.uint64)
    base[1:] = np.cumsum(lens)[:-1]
    host = np.frombuffer(b"".join(streams) + b"\0", dtype=np.uint8).copy()
    g = np.full(k, 64, dtype=np.uint64)  # small slot guesses: OUT_OF_SPACE rounds too
    max_frames = int(lens.sum()) // 2 + k + 16
    f_off = np.zeros(max_frames, dtype=np.uint64)
    f_len = np.zeros(max_frames, dtype=np.uint64)
    f_conn = np.zeros(max_frames, dtype=np.uint32)
    cons = np.zeros(k, dtype=np.uint64)
    st = np.zeros(k, dtype=np.int32)
    nf = ctypes.c_uint32(0)
    rc = cp.lib().capnp_packed_frame_connections(
        host.ctypes.data, int(lens.sum()), base.ctypes.data, lens.ctypes.data, k, g.ctypes.data, frames.ctypes.data,
        frames.size, f_off.ctypes.data, f_len.ctypes.data, f_conn.ctypes.data, max_frames, cons.ctypes.data,
        st.ctypes.data, ctypes.byref(nf))
    assert rc == cp.OK, cp.lib().capnp_packed_last_error()
    n = nf.value
    out = [[] for _ in range(k)]
    for i in range(n):  # pop order within a connection is the table's order
        o, ln, c = int(f_off[i]), int(f_len[i]), int(f_conn[i])
        out[c].append(bytes(frames[o:o + ln]))
    return out, cons.tolist(), st.tolist()


def test_frame_connections_into_page_locked_frames():
    """The frames of every round go D2H on a copy stream while the next round decodes (double-
    buffered slots, capnp_packed_abi.cpp); into a page-locked buffer those copies are truly
    asynchronous. The call must still return with every frame in place: same frames, consumed
    counts and statuses as into a pageable buffer, and as the oracle reader."""
    rng = np.random.default_rng(0xF7A3E)
    streams, expect = [], []
    for c in range(96):
        msgs, packed = make_stream(rng, int(rng.integers(0, 12)))
        data = b"".join(packed)
        if c % 7 == 3 and len(data) > 4:
            data = data[:-3]  # ends inside a message: EndOfStream, the tail stays buffered
        streams.append(data)
        expect.append(oracle_frames(data))
    cap = 4 * sum(len(s) for s in streams) + (1 << 20)
    pinned = torch.empty(cap, dtype=torch.uint8, pin_memory=True).numpy()
    pinned[:] = 0xA5
    pageable = np.full(cap, 0x5A, dtype=np.uint8)
    got_pin = _frame_connections(streams, pinned)
    got_page = _frame_connections(streams, pageable)
    assert got_pin == got_page
    frames, cons, sts = got_pin
    for c, (ofr, rest, code) in enumerate(expect):
        assert frames[c] == ofr, f"connection {c}"
        assert cons[c] == len(streams[c]) - len(rest), f"connection {c}"
        assert sts[c] == (cp.END_OF_STREAM if code in (cp.OK, cp.END_OF_STREAM) else code), f"connection {c}"


def _big_message(rng, words):
    """A one-segment framed message of `words` words (segment table + body), ~50% zero bytes."""
    body = rng.integers(1, 256, 8 * (words - 1), dtype=np.uint8)
    body[rng.random(body.size) < 0.5] = 0
    return pyref.frame([body.tobytes()])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("words", [2 * 1024 * 1024, 8 * 1024 * 1024 + 1],
                         ids=["16MiB", "8Mi_words"])
def test_split_message_in_64k_reads(words):
    """Verdict r3 item 2 (framing.zig:42-90 keeps expected_total across pushes; reader.zig:84-156
    is one pass): a 16 MiB message and one of the 8 Mi-word limit (framing.zig:5), each followed
    by a small one, arrive in 64 KiB socket reads. PackedConnections (beside a second connection
    of small messages) and PackedFramer pop them bit-exact against the oracle reader, and every
    stream byte crosses PCIe once (uploaded_bytes == the stream)."""
    rng = np.random.default_rng(words)
    big = _big_message(rng, words)
    st, pbig = oracle.pack(big)
    assert st == oracle.OK
    msgs, packed = make_stream(rng, 3)
    stream = pbig + packed[0]
    exp0 = oracle_frames(stream)
    assert exp0[0] == [big, msgs[0]] and exp0[2] == cp.OK
    small = b"".join(packed[1:])
    reads = [stream[i:i + 65536] for i in range(0, len(stream), 65536)]
    conns = cp.PackedConnections(2)
    got0, got1 = [], []
    for r, piece in enumerate(reads):
        rd = {0: piece}
        if r < len(small):
            rd[1] = small[r:r + 1]  # the other connection trickles one byte per read
        res = conns.handle_read(rd)
        assert not any(isinstance(v, cp.PackedError) for v in res.values())
        got0 += [bytes(f) for f in res.get(0, [])]
        got1 += [bytes(f) for f in res.get(1, [])]
        if got0 == []:
            assert conns.framers[0].buffered_bytes() == sum(len(x) for x in reads[:r + 1])
    res = conns.handle_read({1: small[len(reads):]})
    got1 += [bytes(f) for f in res.get(1, [])]
    assert got0 == [big, msgs[0]] and got1 == msgs[1:]
    assert conns.framers[0].buffered_bytes() == 0 and conns.framers[1].buffered_bytes() == 0
    stats = conns.session.stats()
    assert stats["uploaded_bytes"] == len(stream) + len(small)
    assert stats["moved_bytes"] <= 2 * len(pbig)  # region doublings: each byte moves O(1) times

    f = cp.PackedFramer()
    out, pushed = [], 0
    for piece in reads:
        f.push(piece)
        pushed += len(piece)
        while (fr := f.pop_frame()) is not None:
            out.append(fr)
        if not out:  # the big message is not whole yet: every pushed byte is held
            assert f.buffered_bytes() == pushed
    assert out == [big, msgs[0]] and f.buffered_bytes() == 0
    assert f.session.stats()["uploaded_bytes"] == len(stream)


def test_framer_session_errors_and_reset():
    """capnp_packed_framer_* through the C-ABI: a bad header after a good message (the good one
    is popped, the error drops the rest), a message overshooting its framed length
    (InvalidPackedMessage), reset and reuse of the connection, and a frames buffer too small
    (OUT_OF_SPACE: the popped frames are valid, the next call pops the rest)."""
    import ctypes
    rng = np.random.default_rng(0xFA11)
    msgs, packed = make_stream(rng, 6)
    bad = bytes([0x03, 0x57, 0x02])  # 600 segments
    # a one-segment header of 1 word whose record then produces 3 zero words: overshoot
    over = bytes([0x10, 0x01, 0x00, 0x02])  # header word 00000000 01000000, then 00 02
    rc, _, _ = oracle.read_packed_message(over, cap=1 << 20)
    assert ORACLE_TO_ABI[rc] == cp.INVALID_PACKED_MESSAGE
    sess = cp.FramerSession(3)
    fr, st = sess.read({0: packed[0] + bad + packed[1], 1: over, 2: packed[2][:5]})
    assert [bytes(x) for x in fr.get(0, [])] == [msgs[0]] and int(st[0]) == cp.SEGMENT_COUNT_LIMIT_EXCEEDED
    assert int(st[1]) == cp.INVALID_PACKED_MESSAGE and int(st[2]) == cp.END_OF_STREAM
    assert sess.buffered(0) == 0 and sess.buffered(1) == 0 and sess.buffered(2) == 5
    sess.reset(2)
    assert sess.buffered(2) == 0
    fr, st = sess.read({0: packed[3], 2: packed[2]})
    assert [bytes(x) for x in fr[0]] == [msgs[3]] and [bytes(x) for x in fr[2]] == [msgs[2]]
    # frames buffer too small: OUT_OF_SPACE with the frames that fit, then the rest
    data = packed[4] + packed[5]
    host = np.frombuffer(data, dtype=np.uint8).copy()
    off = np.zeros(3, dtype=np.uint64)
    ln = np.array([len(data), 0, 0], dtype=np.uint64)
    buf = np.zeros(len(msgs[4]) + 8, dtype=np.uint8)
    fo, fl = np.zeros(4, dtype=np.uint64), np.zeros(4, dtype=np.uint64)
    fc, stc = np.zeros(4, dtype=np.uint32), np.zeros(3, dtype=np.int32)
    nf = ctypes.c_uint32(0)
    L = cp.lib()
    rc = L.capnp_packed_framer_read(sess.handle, host.ctypes.data, len(data), off.ctypes.data, ln.ctypes.data,
                                    buf.ctypes.data, buf.size, fo.ctypes.data, fl.ctypes.data, fc.ctypes.data, 4,
                                    stc.ctypes.data, ctypes.byref(nf))
    assert rc == cp.OUT_OF_SPACE and nf.value == 1
    assert buf[int(fo[0]):int(fo[0]) + int(fl[0])].tobytes() == msgs[4]
    fr, st = sess.read({})
    assert [bytes(x) for x in fr[0]] == [msgs[5]] and sess.buffered(0) == 0
    sess.close()


def _shaped_message(rng, kind):
    """Messages whose packed form stresses the framer walk: many segments (a header of up to 129
    words, decoded across several reads), zero-heavy (2 packed bytes per 256 words), literal-heavy
    (FF runs of 256 words), and ordinary ones."""
    if kind == 0:
        return pyref.frame([bytes(8 * int(rng.integers(0, 3))) for _ in range(int(rng.integers(60, 257)))])
    if kind == 1:
        return pyref.frame([bytes(8 * int(rng.integers(256, 6000)))])
    if kind == 2:
        b = rng.integers(1, 256, 8 * int(rng.integers(200, 3000))).astype(np.uint8)
        return pyref.frame([b.tobytes()])
    return random_message(rng)


def test_framer_session_fuzz_reads():
    """The device-resident session (capnp_packed_framer_*) over 24 connections for 30 rounds:
    each connection's stream cut into reads of 1-7 bytes (headers split byte by byte), ~1 KiB or
    up to 64 KiB, some rounds skipping a connection; regions regrow and the arena is rebuilt as
    connections fall behind. Every frame, in order, against the oracle reader, every byte
    uploaded once."""
    rng = np.random.default_rng(0x5E55)
    n = 24
    streams, expect = [], []
    for c in range(n):
        msgs = [_shaped_message(rng, int(rng.integers(0, 4))) for _ in range(int(rng.integers(1, 6)))]
        data = b"".join(oracle.pack(m)[1] for m in msgs)
        streams.append(data)
        expect.append(msgs)
    size = [int(rng.choice([4, 1024, 65536])) for _ in range(n)]
    pos = [0] * n
    sess = cp.FramerSession(n)
    got = [[] for _ in range(n)]
    uploaded = 0
    for r in range(30):
        reads = {}
        for c in range(n):
            if pos[c] >= len(streams[c]) or (r < 29 and rng.random() < 0.2):
                continue
            k = int(rng.integers(1, size[c] + 1))
            if r == 29:
                k = len(streams[c])  # the last round delivers the rest
            reads[c] = streams[c][pos[c]:pos[c] + k]
            pos[c] += len(reads[c])
            uploaded += len(reads[c])
        fr, st = sess.read(reads)
        assert (st == cp.END_OF_STREAM).all(), st
        for c, frames in fr.items():
            got[c] += [bytes(x) for x in frames]
    for c in range(n):
        assert got[c] == expect[c], f"connection {c}"
        assert sess.buffered(c) == 0 and sess.expected(c) == 0
    assert sess.stats()["uploaded_bytes"] == uploaded == sum(len(s) for s in streams)
    sess.close()


def test_framer_session_many_messages_per_read():
    """One read holding more messages than a walk pass finds per connection (64): the pass
    repeats from where it stopped. Connections with 200 empty messages (2 packed bytes each),
    130 ordinary ones, 70 then a bad header (the 70 are popped, then the error), exactly 64,
    and 65 plus part of a 66th (popped once the rest arrives). Then a frame table of 50 entries
    over 150 messages: three calls (two OUT_OF_SPACE) pop them in order."""
    import ctypes
    rng = np.random.default_rng(0x64D5)
    empty = pyref.frame([b""])
    m0 = [empty] * 200
    m1 = [random_message(rng) for _ in range(130)]
    m2 = [random_message(rng) for _ in range(70)]
    m3 = [random_message(rng) for _ in range(64)]
    m4 = [random_message(rng) for _ in range(66)]
    pk = lambda ms: b"".join(oracle.pack(m)[1] for m in ms)
    bad = bytes([0x03, 0x57, 0x02])  # 600 segments
    tail = oracle.pack(m4[65])[1]
    sess = cp.FramerSession(5)
    fr, st = sess.read({0: pk(m0), 1: pk(m1), 2: pk(m2) + bad + pk(m3[:2]), 3: pk(m3), 4: pk(m4[:65]) + tail[:3]})
    got = {c: [bytes(x) for x in v] for c, v in fr.items()}
    assert got[0] == m0 and got[1] == m1 and got[2] == m2 and got[3] == m3 and got[4] == m4[:65]
    assert [int(x) for x in st] == [cp.END_OF_STREAM, cp.END_OF_STREAM, cp.SEGMENT_COUNT_LIMIT_EXCEEDED,
                                    cp.END_OF_STREAM, cp.END_OF_STREAM]
    assert sess.buffered(4) == 3 and sess.buffered(2) == 0
    fr, st = sess.read({4: tail[3:]})
    assert [bytes(x) for x in fr[4]] == [m4[65]] and (st == cp.END_OF_STREAM).all()
    # a frame table of 50 entries over 150 messages of one connection
    ms = [random_message(rng) for _ in range(150)]
    data = pk(ms)
    host = np.frombuffer(data, dtype=np.uint8).copy()
    off = np.zeros(5, dtype=np.uint64)
    ln = np.array([len(data), 0, 0, 0, 0], dtype=np.uint64)
    buf = np.zeros(sum(len(m) for m in ms) + 64, dtype=np.uint8)
    fo, fl = np.zeros(50, dtype=np.uint64), np.zeros(50, dtype=np.uint64)
    fc, stc = np.zeros(50, dtype=np.uint32), np.zeros(5, dtype=np.int32)
    nf = ctypes.c_uint32(0)
    L = cp.lib()
    out, first, calls = [], True, 0
    while True:
        rc = L.capnp_packed_framer_read(sess.handle, host.ctypes.data if first else None, len(data) if first else 0,
                                        off.ctypes.data if first else None, ln.ctypes.data if first else None,
                                        buf.ctypes.data, buf.size, fo.ctypes.data, fl.ctypes.data, fc.ctypes.data,
                                        50, stc.ctypes.data, ctypes.byref(nf))
        first, calls = False, calls + 1
        assert rc in (cp.OK, cp.OUT_OF_SPACE) and (fc[:nf.value] == 0).all()
        out += [buf[int(fo[i]):int(fo[i]) + int(fl[i])].tobytes() for i in range(nf.value)]
        if rc == cp.OK:
            break
    assert out == ms and calls == 3 and sess.buffered(0) == 0
    sess.close()


def test_framer_readv_threaded_gather_and_arguments():
    """capnp_packed_framer_readv: 96 connections holding ~8 MiB of packed messages in all (the
    threaded gather, by byte range across connection boundaries), a connection with a NULL
    pointer and length 0, a connection whose read ends inside a message; frames bit-exact
    against the messages; a NULL pointer with a length is INVALID_ARGUMENT."""
    import ctypes
    rng = np.random.default_rng(0x7EAD)
    n = 96
    expect, reads = {}, {}
    for c in range(n):
        if c == 5:
            continue  # no bytes: NULL pointer, length 0
        msgs = [pyref.frame([rng.integers(0, 256, 8 * int(rng.integers(500, 3000))).astype(np.uint8).tobytes()])
                for _ in range(int(rng.integers(4, 12)))]
        data = b"".join(oracle.pack(m)[1] for m in msgs)
        if c == 7:
            data += oracle.pack(msgs[0])[1][:100]  # a partial message stays buffered
        expect[c], reads[c] = msgs, data
    total = sum(len(d) for d in reads.values())
    assert total > 4 << 20
    sess = cp.FramerSession(n)
    parts, status = sess.readv_raw(reads)
    got = {}
    for buf, fo, fl, fc in parts:
        for o, ln, c in zip(fo.tolist(), fl.tolist(), fc.tolist()):
            got.setdefault(c, []).append(buf[o:o + ln].tobytes())
    assert got == expect and (status == cp.END_OF_STREAM).all()
    assert sess.buffered(7) == 100 and sess.buffered(5) == 0
    ptrs = (ctypes.c_char_p * n)()
    lens = np.zeros(n, dtype=np.uint64)
    lens[3] = 10  # bytes claimed behind a NULL pointer
    buf = np.zeros(64, dtype=np.uint8)
    fo, fl = np.zeros(4, dtype=np.uint64), np.zeros(4, dtype=np.uint64)
    fc, stc = np.zeros(4, dtype=np.uint32), np.zeros(n, dtype=np.int32)
    nf = ctypes.c_uint32(0)
    rc = cp.lib().capnp_packed_framer_readv(sess.handle, ptrs, lens.ctypes.data, buf.ctypes.data, buf.size,
                                            fo.ctypes.data, fl.ctypes.data, fc.ctypes.data, 4, stc.ctypes.data,
                                            ctypes.byref(nf))
    assert rc == cp.INVALID_ARGUMENT and nf.value == 0
    assert sess.buffered(7) == 100  # nothing appended
    sess.close()


def test_framer_session_steady_stream_reuses_regions():
    """A long-lived session fed 40 reads per connection, each read carrying whole messages plus
    the start of the next one: a connection's held tail slides to its region's start when the
    next read would pass the region's end (no new region, no arena rebuild), so the bytes moved
    stay a small fraction of the stream. Every frame, in order, against the messages."""
    rng = np.random.default_rng(0x57EA)
    n = 8
    msgs = [[random_message(rng) for _ in range(120)] for _ in range(n)]
    streams = [b"".join(oracle.pack(m)[1] for m in ms) for ms in msgs]
    sess = cp.FramerSession(n)
    got = [[] for _ in range(n)]
    pos = [0] * n
    for r in range(40):
        reads = {}
        for c in range(n):
            k = len(streams[c]) - pos[c] if r == 39 else int(rng.integers(1, 3 * len(streams[c]) // 40))
            reads[c] = streams[c][pos[c]:pos[c] + k]
            pos[c] += len(reads[c])
        fr, st = sess.read(reads)
        assert (st == cp.END_OF_STREAM).all()
        for c, v in fr.items():
            got[c] += [bytes(x) for x in v]
    assert got == msgs
    stats = sess.stats()
    total = sum(len(s) for s in streams)
    assert stats["uploaded_bytes"] == total and stats["moved_bytes"] < total // 4, stats
    sess.close()


def test_framer_sessions_release_their_stream_context():
    """a framer session's decode passes run on the session's own stream, so the
    library keeps a context (side stream, events, class queue) for that stream. Destroying the
    session must drop it: 24 sessions created, read (each decodes whole messages) and closed
    leave the library's context count where it was."""
    rng = np.random.default_rng(0x5E55)
    msgs, packed = make_stream(rng, 6)
    stream = b"".join(packed)
    torch.cuda.synchronize()
    before = cp.stream_contexts()
    for _ in range(24):
        sess = cp.FramerSession(2)
        fr, st = sess.read({0: stream, 1: stream[:len(stream) // 2]})
        assert [bytes(x) for x in fr[0]] == msgs
        sess.close()
    assert cp.stream_contexts() == before
