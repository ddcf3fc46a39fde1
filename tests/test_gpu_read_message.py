"""GPU parity of the batched Reader.readPackedMessage (reader.zig:84-156) against
the oracle's restatement (oracle/packed_oracle.c oracle_read_packed_message).

Every case is a reader stream (one unit) holding a packed message, possibly
followed by the next message or cut short. The device result (status, framed
bytes, consumed) must equal the oracle's; errors consume nothing on the device
(the reference's stream position after an error is not observable).
"""
import random
import struct

import numpy as np
import pytest

import capnp_packed as cp
import oracle
import pyref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda"
# oracle return code -> C-ABI status
ORACLE_TO_ABI = {0: cp.OK, -1: cp.END_OF_STREAM, -2: cp.INVALID_SEGMENT_COUNT,
                 -3: cp.SEGMENT_COUNT_LIMIT_EXCEEDED, -6: cp.MESSAGE_TOO_LARGE, -7: cp.INVALID_PACKED_MESSAGE}


def expected(stream: bytes):
    rc, framed, used = oracle.read_packed_message(stream, cap=1 << 20)
    return ORACLE_TO_ABI[rc], (framed if rc == 0 else b""), (used if rc == 0 else 0)


def t64(xs):
    return torch.tensor(list(xs), dtype=torch.int64, device=DEV)


def gpu_read(streams, caps=None, pad_front=0, align=1):
    offs, pos = [], pad_front
    for s in streams:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        pos += len(s)
    host = np.zeros(pos + 32, dtype=np.uint8)
    for o, s in zip(offs, streams):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    d_in = torch.from_numpy(host).to(DEV)
    n = len(streams)
    if caps is None:
        caps = [max(64, len(expected(s)[1])) for s in streams]
    ooffs, opos = [], 0
    for c in caps:
        ooffs.append(opos)
        opos += (c + 15) // 16 * 16
    d_out = torch.zeros(opos + 16, dtype=torch.uint8, device=DEV)
    out_len = torch.full((n,), 7, dtype=torch.int64, device=DEV)
    used = torch.full((n,), 7, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.read_message_batch(d_in, t64(offs), t64(len(s) for s in streams), d_out, t64(ooffs), t64(caps), out_len,
                          used, status)
    torch.cuda.synchronize()
    h = d_out.cpu().numpy()
    lens, sts, us = out_len.cpu().numpy(), status.cpu().numpy(), used.cpu().numpy()
    res = []
    for i in range(n):
        data = h[ooffs[i]:ooffs[i] + lens[i]].tobytes() if sts[i] == cp.OK else b""
        res.append((int(sts[i]), data, int(us[i])))
    return res


def check(streams, **kw):
    got = gpu_read(streams, **kw)
    for i, s in enumerate(streams):
        exp = expected(s)
        assert got[i] == exp, f"stream {i} ({len(s)} B): got status {got[i][0]} used {got[i][2]}, " \
                              f"oracle {exp[0]} used {exp[2]}"


def random_message(rng, max_segs=4, max_words=64, p_zero=0.5):
    segs = []
    for _ in range(rng.randint(1, max_segs)):
        w = rng.randint(0, max_words)
        segs.append(bytes(0 if rng.random() < p_zero else rng.randint(1, 255) for _ in range(8 * w)))
    return segs


def test_reader_kats():
    """reader.zig:304-386."""
    p = bytearray(10)
    p[0] = 0xFF
    p[1:9] = struct.pack("<Q", 0x00000000FFFFFFFF)
    bad_count = bytes(p)
    p[1:9] = struct.pack("<Q", (8 * 1024 * 1024 + 1) << 32)
    too_large = bytes(p)
    streams = [bad_count, too_large, b"\x00\x01", b"\x00", b"\xff", b"\x01", b"\x10\x01\x00\x00", b""]
    got = gpu_read(streams, caps=[64] * len(streams))
    assert [g[0] for g in got] == [cp.INVALID_SEGMENT_COUNT, cp.MESSAGE_TOO_LARGE, cp.INVALID_PACKED_MESSAGE,
                                   cp.END_OF_STREAM, cp.END_OF_STREAM, cp.END_OF_STREAM, cp.OK, cp.END_OF_STREAM]
    assert got[6] == (cp.OK, bytes(4) + b"\x01" + bytes(11), 4)
    check(streams, caps=[64] * len(streams))


def test_single_buffer_mirror():
    segs = [b"packed-stream\x00\x00\x00", bytes(8)]
    a = pyref.to_packed_bytes(segs)
    b = pyref.to_packed_bytes([bytes(range(1, 17))])
    framed, used = cp.read_packed_message_bytes(a + b)
    assert framed == pyref.frame(segs) and used == len(a)
    import io
    f = io.BytesIO(a + b)
    assert cp.Reader.read_packed_message(f) == pyref.frame(segs)
    assert cp.Reader.read_packed_message(f) == pyref.frame([bytes(range(1, 17))])
    with pytest.raises(cp.EndOfStream):
        cp.Reader.read_packed_message(f)
    with pytest.raises(cp.InvalidPackedMessage):
        cp.Reader.read_packed_message(b"\x00\x01")
    # a zero-run message far larger than the first capacity guess (8 x packed length)
    big = pyref.to_packed_bytes([bytes(8 * 4000)])
    framed, used = cp.read_packed_message_bytes(big)
    assert framed == pyref.frame([bytes(8 * 4000)]) and used == len(big)


def test_concatenated_streams_message_by_message():
    """Each unit holds several messages back to back; read them one call at a time,
    advancing every reader by its consumed count (the socket-reader loop)."""
    rng = random.Random(0xFEDCBA98)
    n_units, per = 96, 5
    msgs = [[random_message(rng, p_zero=rng.choice([0.1, 0.5, 0.9])) for _ in range(per)] for _ in range(n_units)]
    streams = [b"".join(pyref.to_packed_bytes(m) for m in ms) for ms in msgs]
    pos = [0] * n_units
    for k in range(per + 1):
        rest = [s[p:] for s, p in zip(streams, pos)]
        got = gpu_read(rest)
        for i in range(n_units):
            exp = expected(rest[i])
            assert got[i] == exp, f"unit {i}, message {k}"
            if k < per:
                assert got[i][0] == cp.OK and got[i][1] == pyref.frame(msgs[i][k])
            else:
                assert got[i][0] == cp.END_OF_STREAM
            pos[i] += got[i][2]


def test_truncations_and_trailing_bytes():
    rng = random.Random(7)
    streams = []
    for _ in range(24):
        a = pyref.to_packed_bytes(random_message(rng, max_words=40))
        nxt = pyref.to_packed_bytes(random_message(rng, max_words=8))
        for cut in sorted(set([0, 1, 2, len(a) // 2, len(a) - 1, len(a)] + [rng.randrange(len(a) + 1)])):
            streams.append(a[:cut])
        streams.append(a + nxt[:3])
        streams.append(a + b"\xff")
    check(streams)


def test_many_segment_headers():
    """Headers spanning many records: 511/512 segments (limit), 513 (over the limit),
    an even count (padding word), and sizes summing past 8 Mi words."""
    rng = random.Random(11)
    streams = []
    for count in (1, 2, 7, 64, 255, 511, 512):
        segs = [bytes(8 * rng.randint(0, 2)) if rng.random() < 0.5 else bytes(rng.randint(1, 255) for _ in range(8))
                for _ in range(count)]
        streams.append(pyref.to_packed_bytes(segs))
    over = struct.pack("<I", 512) + b"".join(struct.pack("<I", 1) for _ in range(513))
    over += bytes((-len(over)) % 8) + bytes(8 * 513)
    streams.append(pyref.pack(over))  # 513 segments -> SegmentCountLimitExceeded
    huge = struct.pack("<II", 1, 5 * 1024 * 1024) + struct.pack("<II", 4 * 1024 * 1024, 0)
    streams.append(pyref.pack(huge))  # 9 Mi words -> MessageTooLarge before the body is read
    check(streams, caps=[1 << 16] * len(streams))
    assert gpu_read(streams[-2:], caps=[64, 64])[0][0] == cp.SEGMENT_COUNT_LIMIT_EXCEEDED


def test_large_messages_take_the_full_path():
    """Messages whose packed size exceeds the fill pass's window (> 5 KB) and slots too
    small for the index records go through the wave decoder; OUT_OF_SPACE reports the
    framed length and the packed length."""
    rng = random.Random(3)
    streams, caps = [], []
    for words in (700, 2000, 9000):
        segs = [bytes(0 if rng.random() < 0.3 else rng.randint(1, 255) for _ in range(8 * words))]
        s = pyref.to_packed_bytes(segs) + pyref.to_packed_bytes([bytes(16)])
        streams.append(s)
        caps.append(len(pyref.frame(segs)))
    check(streams, caps=caps)
    small = gpu_read(streams, caps=[64] * len(streams))
    for i, s in enumerate(streams):
        st, framed, used = expected(s)
        assert small[i][0] == cp.OUT_OF_SPACE and small[i][2] == used


def test_fuzz_against_oracle():
    """message_test.zig:1076-1093 style random buffers, read as streams."""
    rng = random.Random(0xA7C41E59F0328D6B)
    streams = []
    for _ in range(1024):
        n = rng.randrange(160)
        b = bytearray(rng.getrandbits(8) for _ in range(n))
        if n and rng.random() < 0.5:
            b[0] = rng.choice([0x00, 0xFF, 0x10, 0x01])
        streams.append(bytes(b))
    check(streams, pad_front=3)


def test_framed_units_at_scale():
    """64K framed 4-KiB messages (1 segment of 511 words, p = 0.5), encoded on device
    into slots and read back message by message from the slots."""
    n, ub = 1 << 16, 4096
    d_in = cp.generate(n, ub, seed=0xC0DE0002, zero_thresh=128)
    d_in.view(torch.int64).view(n, ub // 8)[:, 0] = (ub // 8 - 1) << 32  # header: 1 segment, 511 words
    in_off, in_len = cp.uniform_layout(n, ub)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot)
    d_pk = torch.zeros(n * slot, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.zeros(n, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    # each reader holds its message plus the slot's tail (bytes of no message)
    d_out = torch.zeros(n * ub, dtype=torch.uint8, device=DEV)
    olen = torch.zeros(n, dtype=torch.int64, device=DEV)
    used = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.zeros(n, dtype=torch.int32, device=DEV)
    tail = torch.minimum(plen + 7, pk_cap)
    cp.read_message_batch(d_pk, pk_off, tail, d_out, in_off, in_len, olen, used, st)
    torch.cuda.synchronize()
    assert (st == 0).all() and torch.equal(used, plen) and (olen == ub).all()
    assert torch.equal(d_out, d_in)


def test_single_buffer_unbounded_cap():
    # cap = SIZE_MAX (a C caller's "unbounded" idiom): the device slot is sized by what
    # reader.zig can produce, so the workspace sums cannot wrap and nothing is written
    # past the framed message
    import ctypes
    segs = [bytes(range(1, 41)), bytes(16)]
    a = pyref.to_packed_bytes(segs)
    exp = pyref.frame(segs)
    src = ctypes.create_string_buffer(a, len(a))
    out = ctypes.create_string_buffer(len(exp) + 64)
    ctypes.memset(out, 0xAB, len(exp) + 64)
    n, used = ctypes.c_size_t(), ctypes.c_size_t()
    st = cp.lib().capnp_packed_read_message(src, len(a), out, ctypes.c_size_t(-1).value, ctypes.byref(n),
                                            ctypes.byref(used))
    assert st == cp.OK and n.value == len(exp) and used.value == len(a)
    assert out.raw[:len(exp)] == exp and out.raw[len(exp):] == b"\xab" * 64


def _overshoot_stream(rng, body_words, tail):
    """A one-segment message of body_words words whose packed body ends with `tail`: a record
    that ends exactly at the framed length, or a zero / literal run that passes it (its
    literal bytes whole or cut), so the reader stops inside a run (reader.zig:146-153)."""
    head = pyref.pack(struct.pack("<II", 0, body_words))
    body = bytearray()
    words = 0
    room = body_words - 2
    while words < room:
        t = rng.randrange(1, 255)
        body += bytes([t]) + bytes(rng.randrange(1, 256) for _ in range(bin(t).count("1")))
        words += 1
    if tail == "exact":
        body += b"\x00\x01"                      # two zero words: ends at the framed length
    elif tail == "zero_run_over":
        body += bytes([0, rng.randrange(2, 40)])  # passes it inside a zero run
    else:
        c = rng.randrange(2, 40)
        lit = bytes(rng.randrange(256) for _ in range(8 * c))
        if tail == "literal_cut":
            lit = lit[:rng.randrange(len(lit))]
        body += b"\xff" + bytes(rng.randrange(256) for _ in range(8)) + bytes([c]) + lit
    return bytes(head) + bytes(body) + bytes(rng.randrange(256) for _ in range(rng.randrange(0, 24)))


def test_overshoot_inside_runs_and_the_words_bound():
    """Messages of 1020 .. 1030 framed words (kRdWordsMax = 1024 on the words decoder, longer ones
    on the walk passes), each ending exactly, or passing the framed length inside a zero run, a
    whole literal run (InvalidPackedMessage) or a cut literal run (EndOfStream), at every
    alignment of the stream; status, framed bytes and consumed against the oracle."""
    rng = random.Random(0x0E5)
    streams = []
    for body_words in range(1019, 1030):
        for tail in ("exact", "zero_run_over", "literal_over", "literal_cut"):
            streams.append(_overshoot_stream(rng, body_words, tail))
    got_codes = set()
    for pad in range(0, 16, 3):
        check(streams, pad_front=pad, caps=[9000] * len(streams))
        got_codes |= {expected(s)[0] for s in streams}
    assert got_codes == {cp.OK, cp.INVALID_PACKED_MESSAGE, cp.END_OF_STREAM}
    # slots 8 B short: OUT_OF_SPACE with the framed length and the packed length
    ok = [s for s in streams if expected(s)[0] == cp.OK]
    short = gpu_read(ok, caps=[len(expected(s)[1]) - 8 for s in ok])
    for s, g in zip(ok, short):
        st, framed, used = expected(s)
        assert g[0] == cp.OUT_OF_SPACE and g[2] == used
