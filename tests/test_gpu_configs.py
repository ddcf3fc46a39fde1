"""GPU parity on SURVEY §8(d)'s configs C1 and C5 (C2-C4 shapes are in
test_gpu_parity.py / test_sharding.py).

C1: the reference's CPU bench shape made concrete as SURVEY asks: one framed message
    of 64 segments x 1 KiB (p = 0.5) behind a valid segment table, packed through the
    single-buffer C-ABI (MessageBuilder.toPackedBytes, message.zig:2175-2179) and read
    back (Message.initPacked, message.zig:400-408), bit-exact against the oracle.
C5: skewed unit sizes (truncated Pareto, alpha = 1.1, 64 B .. 256 KiB) in one batch,
    including units far beyond the 4-KiB fast-path tile, every unit against the oracle.
"""
import numpy as np
import pytest

import capnp_packed as cp
import oracle
import pyref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


DEV = "cuda"


def c1_segments(seed=0xC0DE0001):
    data = oracle.generate(64, 1024, seed=seed, zero_thresh=128)
    return [data[i * 1024:(i + 1) * 1024].tobytes() for i in range(64)]


def test_c1_64_segment_message_single_buffer():
    segs = c1_segments()
    b = cp.MessageBuilder()
    for s in segs:
        b.create_segment(s)
    framed = b.to_bytes()
    assert framed == pyref.frame(segs) and len(framed) == 8 * 33 + 64 * 1024
    packed = b.to_packed_bytes()
    st, exp = oracle.pack(framed)
    assert st == oracle.OK and packed == exp
    msg = cp.Message.init_packed(packed)
    assert [bytes(s) for s in msg.segments] == segs and msg.backing_data == framed
    assert cp.Reader.read_packed_message(packed + b"\x00") == framed


def test_c1_batch_of_messages(decoder):
    """64 C1 messages (different seeds) through the batch entry points."""
    msgs = [pyref.frame(c1_segments(0xC0DE0100 + k)) for k in range(64)]
    ub = len(msgs[0])
    d_in = torch.from_numpy(np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()).to(DEV)
    n = len(msgs)
    in_off, in_len = cp.uniform_layout(n, ub)
    slot = (cp.encode_bound(ub) + 15) // 16 * 16
    pk_off, pk_cap = cp.uniform_layout(n, slot)
    d_pk = torch.zeros(n * slot, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    d_out = torch.zeros(n * ub, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
    torch.cuda.synchronize()
    pk, lens = d_pk.cpu().numpy(), plen.cpu().numpy()
    for k, m in enumerate(msgs):
        st, exp = oracle.pack(m)
        assert pk[k * slot:k * slot + lens[k]].tobytes() == exp, f"message {k}"
    assert (pst.cpu() == 0).all() and (ust.cpu() == 0).all() and torch.equal(d_out, d_in)


def pareto_sizes(n, seed):
    u = np.random.default_rng(seed).random(n)
    return (8 * np.floor(np.clip(64.0 * (1.0 - u) ** (-1.0 / 1.1), 64, 262144) / 8)).astype(np.int64)


@pytest.mark.parametrize("thr", [26, 128, 230])
def test_c5_skewed_sizes_every_unit(thr, decoder):
    sizes = pareto_sizes(3000, seed=0xC0DE0005 + thr)
    # units around and far beyond the 512-word tile, and both size extremes
    extra = [4088, 4096, 4104, 8192, 12288 + 8, 65536, 262144, 64, 8]
    sizes = np.concatenate([sizes, np.array(extra, dtype=np.int64)])
    n = len(sizes)
    off = np.zeros(n + 1, dtype=np.int64)
    off[1:] = np.cumsum(sizes)
    U = int(off[-1])
    host = oracle.generate(1, U, seed=0xC0DE0005, zero_thresh=thr)
    # long zero and literal runs across tile boundaries in the big units
    big = np.nonzero(sizes >= 8192)[0]
    for j, i in enumerate(big):
        a = int(off[i])
        host[a + 4000:a + 4000 + 3000] = 0 if j % 2 else 0x5A
    d_in = torch.from_numpy(host).to(DEV)
    t_off = torch.from_numpy(off[:-1].copy()).to(DEV)
    t_len = torch.from_numpy(sizes).to(DEV)
    caps = (sizes // 8) * 10
    slots = (caps + 15) // 16 * 16
    poff = np.zeros(n, dtype=np.int64)
    poff[1:] = np.cumsum(slots)[:-1]
    d_pk = torch.zeros(int(slots.sum()) + 16, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    t_poff = torch.from_numpy(poff).to(DEV)
    cp.encode_batch(d_in, t_off, t_len, d_pk, t_poff, torch.from_numpy(caps).to(DEV), plen, pst)
    d_out = torch.zeros(U + 16, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, t_poff, plen, d_out, t_off, t_len, ulen, ust)
    torch.cuda.synchronize()
    pk, lens, sts = d_pk.cpu().numpy(), plen.cpu().numpy(), pst.cpu().numpy()
    for i in range(n):
        st, exp = oracle.pack(host[off[i]:off[i + 1]].tobytes())
        assert sts[i] == cp.OK and pk[poff[i]:poff[i] + lens[i]].tobytes() == exp, f"unit {i} ({sizes[i]} B)"
    assert (ust.cpu() == 0).all() and torch.equal(ulen, t_len)
    assert np.array_equal(d_out.cpu().numpy()[:U], host)


def test_c5_full_size_1M_units(decoder):
    """BASELINE configs[4] at its stated size: 1M units of truncated-Pareto sizes
    64 B..256 KiB (the bench's seed), p = 0.5. decode(encode(x)) == x on device for
    every unit; every unit over 64 KiB and a strided sample of the rest byte-compared
    with the oracle."""
    n = 1 << 20
    sizes = pareto_sizes(n, seed=0xC0DE0005)
    off = np.zeros(n + 1, dtype=np.int64)
    off[1:] = np.cumsum(sizes)
    U = int(off[-1])
    d_in = cp.generate(1, U, seed=0xC0DE0005, zero_thresh=128, device=DEV)
    t_off = torch.from_numpy(off[:-1].copy()).to(DEV)
    t_len = torch.from_numpy(sizes).to(DEV)
    caps = (sizes // 8) * 10
    slots = (caps + 15) // 16 * 16
    poff = np.zeros(n, dtype=np.int64)
    poff[1:] = np.cumsum(slots)[:-1]
    d_pk = torch.zeros(int(slots.sum()) + 16, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    t_poff = torch.from_numpy(poff).to(DEV)
    cp.encode_batch(d_in, t_off, t_len, d_pk, t_poff, torch.from_numpy(caps).to(DEV), plen, pst)
    d_out = torch.zeros(U, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, t_poff, plen, d_out, t_off, t_len, ulen, ust)
    torch.cuda.synchronize()
    assert (pst == 0).all().item() and (ust == 0).all().item()
    assert torch.equal(ulen, t_len) and torch.equal(d_out, d_in)
    host = d_in.cpu().numpy()
    pk, lens = d_pk.cpu().numpy(), plen.cpu().numpy()
    pick = np.union1d(np.nonzero(sizes > 65536)[0], np.arange(0, n, 521))
    for i in pick:
        st, exp = oracle.pack(host[off[i]:off[i + 1]].tobytes())
        assert st == oracle.OK and lens[i] == len(exp) and pk[poff[i]:poff[i] + lens[i]].tobytes() == exp, \
            f"unit {i} ({sizes[i]} B)"


def _encode_units(units):
    offs, pos = [], 0
    for u in units:
        offs.append(pos)
        pos += len(u)
    host = np.zeros(pos + 16, dtype=np.uint8)
    for o, u in zip(offs, units):
        host[o:o + len(u)] = np.frombuffer(u, dtype=np.uint8)
    n = len(units)
    caps = [10 * (len(u) // 8) for u in units]
    poffs, q = [], 0
    for c in caps:
        poffs.append(q)
        q += (c + 15) // 16 * 16
    t = lambda xs: torch.tensor(xs, dtype=torch.int64, device=DEV)  # noqa: E731
    d_out = torch.zeros(q + 16, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(torch.from_numpy(host).to(DEV), t(offs), t([len(u) for u in units]), d_out, t(poffs), t(caps),
                    plen, pst)
    sz = torch.zeros(n, dtype=torch.int64, device=DEV)
    sst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encoded_size_batch(torch.from_numpy(host).to(DEV), t(offs), t([len(u) for u in units]), sz, sst)
    torch.cuda.synchronize()
    h, lens = d_out.cpu().numpy(), plen.cpu().numpy()
    assert (pst.cpu() == 0).all() and (sst.cpu() == 0).all() and torch.equal(sz, plen)
    return [h[poffs[i]:poffs[i] + lens[i]].tobytes() for i in range(n)]


def test_tiled_encode_run_carries():
    """Units past the 512-word tile: zero and literal runs that start before a tile
    boundary and end after it (heads at 256-word steps from the run start), runs
    ending exactly at a tile end, and breaks just past the 256-word lookahead."""
    rng = np.random.default_rng(5)
    lit = lambda k: rng.integers(1, 256, 8 * k, dtype=np.uint8).tobytes()  # noqa: E731
    mixed = lambda k: bytes(rng.integers(0, 256, 8 * k, dtype=np.uint8) * (rng.random(8 * k) < 0.5))  # noqa: E731
    units = []
    for kind in (lambda k: bytes(8 * k), lit):
        for start in (1, 255, 256, 300, 400, 511, 512):
            for length in (1, 255, 256, 257, 600, 1023, 1500):
                units.append(mixed(start) + kind(length) + mixed(64))
        units.append(kind(2048))
        units.append(kind(512) + mixed(1))
        units.append(mixed(511) + kind(1) + mixed(600))
    units.append(bytes(8 * 513))
    units.append(lit(513))
    units.append(mixed(8 * 1024))
    got = _encode_units(units)
    for i, u in enumerate(units):
        st, exp = oracle.pack(u)
        assert got[i] == exp, f"unit {i} ({len(u) // 8} words)"


# ---------------------------------------------------------------------------
# framing fused with the codec
# ---------------------------------------------------------------------------

def _segment_pool(messages, rng):
    """Every segment of every message placed at a shuffled, 8-aligned offset of one
    device pool; returns (pool, seg_ptr, seg_len, seg_first, seg_count)."""
    flat = [s for m in messages for s in m]
    order = rng.permutation(len(flat)) if flat else np.zeros(0, dtype=np.int64)
    offs = [0] * len(flat)
    pos = 0
    for k in order:
        pos += 8 * int(rng.integers(0, 3))  # gaps between segments
        offs[k] = pos
        pos += len(flat[k])
    host = np.zeros(pos + 16, dtype=np.uint8)
    for o, s in zip(offs, flat):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    pool = torch.from_numpy(host).to(DEV)
    base = pool.data_ptr()
    seg_ptr = torch.tensor([base + o for o in offs] or [0], dtype=torch.int64, device=DEV)
    seg_len = torch.tensor([len(s) for s in flat] or [0], dtype=torch.int64, device=DEV)
    first, k = [], 0
    for m in messages:
        first.append(k)
        k += len(m)
    return (pool, seg_ptr, seg_len, torch.tensor(first, dtype=torch.int32, device=DEV),
            torch.tensor([len(m) for m in messages], dtype=torch.int32, device=DEV))


def _frame(segs):
    return pyref.frame(segs if segs else [b""])  # toBytes adds one empty segment (message.zig:2128-2130)


def test_encode_message_batch_matches_toPackedBytes():
    rng = np.random.default_rng(17)

    def seg(words, p):
        b = rng.integers(1, 256, 8 * words, dtype=np.uint8)
        b[rng.random(8 * words) < p] = 0
        return b.tobytes()

    messages = [[], [b""], [seg(1, .5)], [seg(0, .5), seg(3, .5)]]
    for _ in range(200):
        p = float(rng.choice([0.1, 0.5, 0.9, 1.0, 0.0]))
        messages.append([seg(int(rng.integers(0, 300)), p) for _ in range(int(rng.integers(1, 12)))])
    messages.append([seg(1, .5) for _ in range(512)])            # the segment limit, header of 257 words
    # around the 64 segments the one-tile pass takes (a segment per lane; more go to the tiled
    # pass), and the 255 offsets an earlier one-tile pass kept in its row pads
    for k in (63, 64, 65, 254, 255, 256, 300):
        messages.append([seg(int(rng.integers(0, 2)), .5) for _ in range(k)])
    messages.append([seg(700, .5), seg(2000, 0.97), seg(5, 0.0)])  # tiles, zero and literal runs across segments
    messages.append([bytes(8 * 600), bytes(8 * 600)])             # one zero run over two segments and tiles
    pool, seg_ptr, seg_len, first, count = _segment_pool(messages, rng)
    n = len(messages)
    caps = [cp.encode_bound(len(_frame(m))) for m in messages]
    offs, q = [], 0
    for c in caps:
        offs.append(q)
        q += (c + 15) // 16 * 16
    t = lambda xs: torch.tensor(xs, dtype=torch.int64, device=DEV)  # noqa: E731
    d_out = torch.zeros(q + 16, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_message_batch(seg_ptr, seg_len, first, count, d_out, t(offs), t(caps), out_len, status)
    sizes = torch.zeros(n, dtype=torch.int64, device=DEV)
    sst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_message_batch(seg_ptr, seg_len, first, count, None, None, None, sizes, sst)
    torch.cuda.synchronize()
    h, lens, sts = d_out.cpu().numpy(), out_len.cpu().numpy(), status.cpu().numpy()
    for i, m in enumerate(messages):
        st, exp = oracle.pack(_frame(m))
        assert st == oracle.OK
        assert sts[i] == cp.OK and h[offs[i]:offs[i] + lens[i]].tobytes() == exp, f"message {i}"
    assert torch.equal(sizes, out_len) and (sst.cpu() == 0).all()


def test_encode_message_batch_stress():
    """The shipped message pass over ~20K varied messages (verdict r4 item 3):
    the one-tile pass (one message per wave: segment table in the row pads, the u8 segment map,
    the pair gather) for most of them, and enough many-segment and multi-tile messages that each
    wave of the grid-striding tiled pass codes dozens. Segment counts straddle the one-tile limit
    (64) and lengths straddle a tile (512 framed words); empty segments, zero and literal runs
    across segment edges, the bench's 4 x 127-word shape, and segments placed in shuffled order
    across one pool. Every message against the oracle, and the size-only pass against the coding
    pass."""
    rng = np.random.default_rng(0x5EED5)
    pat = rng.integers(1, 256, 8 * 4096, dtype=np.uint8)
    pat[rng.random(pat.size) < 0.5] = 0

    def seg(words):
        if words == 0:
            return b""
        kind = rng.integers(0, 4)
        if kind == 0:
            return bytes(8 * words)  # one zero run
        if kind == 1:
            return rng.integers(1, 256, 8 * words, dtype=np.uint8).tobytes()  # literal words
        o = int(rng.integers(0, pat.size // 8 - words)) * 8
        return pat[o:o + 8 * words].tobytes()

    messages = []
    for i in range(20000):
        r = rng.random()
        if r < 0.35:    # the bench's framing shape
            messages.append([seg(127) for _ in range(4)])
        elif r < 0.80:  # one tile, a few segments, some empty
            messages.append([seg(int(rng.choice([0, 1, 2, 17, 60, 120]))) for _ in range(int(rng.integers(0, 9)))])
        elif r < 0.90:  # around the one-tile segment limit
            k = int(rng.choice([62, 63, 64, 65, 66, 100]))
            messages.append([seg(int(rng.integers(0, 5))) for _ in range(k)])
        elif r < 0.97:  # around a tile of framed words
            w = int(rng.choice([505, 508, 509, 510, 511, 512, 513, 600]))
            k = int(rng.integers(1, 4))
            messages.append([seg(w // k) for _ in range(k - 1)] + [seg(w - (k - 1) * (w // k))])
        else:           # several tiles
            messages.append([seg(int(rng.integers(300, 1500))) for _ in range(int(rng.integers(1, 4)))])
    pool, seg_ptr, seg_len, first, count = _segment_pool(messages, rng)
    n = len(messages)
    frames = [_frame(m) for m in messages]
    caps = [cp.encode_bound(len(f)) for f in frames]
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum([(c + 15) // 16 * 16 for c in caps])[:-1]
    total = int(offs[-1]) + (caps[-1] + 15) // 16 * 16
    d_out = torch.zeros(total + 16, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    t_off = torch.from_numpy(offs).to(DEV)
    t_cap = torch.tensor(caps, dtype=torch.int64, device=DEV)
    cp.encode_message_batch(seg_ptr, seg_len, first, count, d_out, t_off, t_cap, out_len, status)
    sizes = torch.zeros(n, dtype=torch.int64, device=DEV)
    sst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_message_batch(seg_ptr, seg_len, first, count, None, None, None, sizes, sst)
    torch.cuda.synchronize()
    h, lens, sts = d_out.cpu().numpy(), out_len.cpu().numpy(), status.cpu().numpy()
    assert (sts == cp.OK).all(), np.flatnonzero(sts != cp.OK)[:10]
    for i, f in enumerate(frames):
        st, exp = oracle.pack(f)
        assert st == oracle.OK
        assert h[offs[i]:offs[i] + lens[i]].tobytes() == exp, f"message {i} ({len(messages[i])} segments)"
    assert torch.equal(sizes, out_len) and (sst.cpu() == 0).all()


def test_encode_message_batch_errors():
    rng = np.random.default_rng(3)
    messages = [[bytes(8)] * 513, [bytes(8), bytes(12)], [bytes(range(1, 65))]]
    pool, seg_ptr, seg_len, first, count = _segment_pool(messages, rng)
    n = len(messages)
    t = lambda xs: torch.tensor(xs, dtype=torch.int64, device=DEV)  # noqa: E731
    d_out = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_message_batch(seg_ptr, seg_len, first, count, d_out, t([0, 1024, 2048]), t([1024, 1024, 20]),
                            out_len, status)
    torch.cuda.synchronize()
    exp_len = len(oracle.pack(_frame(messages[2]))[1])
    assert status.cpu().tolist() == [cp.INVALID_ARGUMENT, cp.INVALID_ARGUMENT, cp.OUT_OF_SPACE]
    assert int(out_len[2]) == exp_len


def test_message_init_batch_matches_message_init():
    rng = np.random.default_rng(23)
    frames = []
    for _ in range(300):
        segs = [bytes(8 * int(rng.integers(0, 20))) for _ in range(int(rng.integers(1, 9)))]
        f = pyref.frame(segs)
        kind = int(rng.integers(0, 6))
        if kind == 1:
            f = f + bytes(8 * int(rng.integers(1, 4)))      # trailing bytes are ignored
        elif kind == 2:
            f = f[:int(rng.integers(0, len(f)))]              # truncated anywhere
        frames.append(f)
    frames += [b"", b"\x00\x00", b"\xff\xff\xff\xff" + bytes(12), struct_u32(512) + bytes(4 * 514 + 8),
               struct_u32(511) + bytes(4 * 513)]
    offs, pos = [], 0
    for f in frames:
        offs.append(pos)
        pos += (len(f) + 7) // 8 * 8
    host = np.zeros(pos + 8, dtype=np.uint8)
    for o, f in zip(offs, frames):
        host[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    n, ms = len(frames), 16
    cnt = torch.zeros(n, dtype=torch.int32, device=DEV)
    so = torch.zeros(n * ms, dtype=torch.int64, device=DEV)
    sl = torch.zeros(n * ms, dtype=torch.int64, device=DEV)
    st = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.message_init_batch(torch.from_numpy(host).to(DEV), torch.tensor(offs, dtype=torch.int64, device=DEV),
                          torch.tensor([len(f) for f in frames], dtype=torch.int64, device=DEV), ms, cnt, so, sl, st)
    torch.cuda.synchronize()
    codes = {0: cp.OK, -1: cp.END_OF_STREAM, -2: cp.INVALID_SEGMENT_COUNT, -3: cp.SEGMENT_COUNT_LIMIT_EXCEEDED,
             -4: cp.TRUNCATED_MESSAGE}
    cnt, so, sl, st = cnt.cpu().numpy(), so.cpu().numpy(), sl.cpu().numpy(), st.cpu().numpy()
    for i, f in enumerate(frames):
        rc, table = oracle.message_init(f, max_segs=ms)
        assert st[i] == codes[rc], f"frame {i}"
        if rc == 0:
            assert cnt[i] == len(table) or (cnt[i] > ms and len(table) == ms)
            got = [(int(so[i * ms + j]), int(sl[i * ms + j])) for j in range(min(int(cnt[i]), ms))]
            assert got == [(int(a), int(b)) for a, b in table], f"frame {i}"


def struct_u32(v):
    return int(v).to_bytes(4, "little")


@pytest.mark.parametrize("flags", [cp.LAUNCH_MID_SIDE_STREAM, cp.LAUNCH_LONG_INLINE,
                                   cp.LAUNCH_MID_SIDE_STREAM | cp.LAUNCH_LONG_INLINE, cp.LAUNCH_CLASS_SCAN],
                         ids=["mid_side_stream", "long_inline", "both", "class_scan"])
def test_c5_launch_flags(flags):
    """The launch policy (capnp_packed_set_launch_flags): the second side
    stream for a decode batch's mid units (the small decoder's grid then at 85%), the long
    units after the main grid instead of on the side stream, and the class pass's scan as its
    own kernel (the path of batches over 1M units; at most 1M, the scatter kernel scans). The
    C5 tests above under each."""
    with cp.launch_flags(flags):
        for thr in (26, 128, 230):
            test_c5_skewed_sizes_every_unit(thr, "twopass")
        test_c5_full_size_1M_units("twopass")
        with cp.decoder("words"):
            test_c5_skewed_sizes_every_unit(128, "words")


def _segment_pool_end_to_end(messages, rng):
    """Each message's segments laid end to end (a MessageBuilder arena's layout), the message's
    first segment at 0 or 8 mod 16 of the pool; returns what _segment_pool returns."""
    offs, pos = [], 0
    for i, m in enumerate(messages):
        pos = (pos + 15) // 16 * 16 + 8 * (i % 2) + 16 * int(rng.integers(0, 3))
        for s in m:
            offs.append(pos)
            pos += len(s)
    flat = [s for m in messages for s in m]
    host = np.zeros(pos + 16, dtype=np.uint8)
    for o, s in zip(offs, flat):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    pool = torch.from_numpy(host).to(DEV)
    base = pool.data_ptr()
    assert base % 16 == 0
    seg_ptr = torch.tensor([base + o for o in offs] or [0], dtype=torch.int64, device=DEV)
    seg_len = torch.tensor([len(s) for s in flat] or [0], dtype=torch.int64, device=DEV)
    first, k = [], 0
    for m in messages:
        first.append(k)
        k += len(m)
    return (pool, seg_ptr, seg_len, torch.tensor(first, dtype=torch.int32, device=DEV),
            torch.tensor([len(m) for m in messages], dtype=torch.int32, device=DEV))


def test_encode_message_segments_end_to_end():
    """The one-tile encoder's end-to-end path (encode_message_tile1_body: one staged run after
    header words computed per lane) against toPackedBytes (message.zig:2123-2179, the oracle):
    1 .. 64 segments (even and odd counts: the padding word), empty segments, bases at 0 and
    8 mod 16, and framed lengths up to and around the one-tile limit of 512 words."""
    rng = np.random.default_rng(0xE2E)

    def seg(words, p):
        b = rng.integers(1, 256, 8 * words, dtype=np.uint8)
        b[rng.random(8 * words) < p] = 0
        return b.tobytes()

    messages = []
    for count in list(range(1, 17)) + [31, 32, 33, 63, 64]:
        for target in (8, 200, 480, 505, 512, 530):  # framed words aimed at around the tile limit
            hw = (1 + count + (0 if count % 2 else 1)) // 2
            room = max(target - hw, 0)
            cuts = np.sort(rng.integers(0, room + 1, count - 1)) if count > 1 else np.zeros(0, dtype=np.int64)
            sizes = np.diff(np.concatenate([[0], cuts, [room]])).astype(int)
            if count > 2:
                sizes[int(rng.integers(0, count))] += sizes[0] if rng.random() < 0.3 else 0
                sizes[0] = 0 if rng.random() < 0.3 else sizes[0]  # empty segments
            p = float(rng.choice([0.1, 0.5, 0.9]))
            messages.append([seg(int(w), p) for w in sizes])
    pool, seg_ptr, seg_len, first, count = _segment_pool_end_to_end(messages, rng)
    n = len(messages)
    caps = [cp.encode_bound(len(_frame(m))) for m in messages]
    offs, q = [], 0
    for c in caps:
        offs.append(q)
        q += (c + 15) // 16 * 16
    t = lambda xs: torch.tensor(xs, dtype=torch.int64, device=DEV)  # noqa: E731
    d_out = torch.zeros(q + 16, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_message_batch(seg_ptr, seg_len, first, count, d_out, t(offs), t(caps), out_len, status)
    torch.cuda.synchronize()
    h, lens, sts = d_out.cpu().numpy(), out_len.cpu().numpy(), status.cpu().numpy()
    one_tile = 0
    for i, m in enumerate(messages):
        st, exp = oracle.pack(_frame(m))
        assert st == oracle.OK
        one_tile += len(_frame(m)) // 8 <= 512
        assert sts[i] == cp.OK and h[offs[i]:offs[i] + lens[i]].tobytes() == exp, f"message {i}: {len(m)} segments"
    assert one_tile >= n // 2
