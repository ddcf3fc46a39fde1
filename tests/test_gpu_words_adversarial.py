"""The words decoder (decode_words_kernel) on arbitrary mid-size packed input,
against the oracle's unpackPacked / estimateUnpackedSize (message.zig:88-191), unit by unit.

Round 5's tests fed the words decoder only encoder output (and truncations of it); random
corpora were all under 160 bytes, so they went to the small-unit kernel. Here every unit is a
mid unit (513 .. 5120 packed bytes), decoded from a dense packed stream at random byte
alignments into 8-B aligned slots with canaries on both sides:
- random bytes (arbitrary tags and counts: mostly UNEXPECTED_EOF, some OK / OUT_OF_SPACE);
- valid record streams with one tag or count byte replaced;
- record streams rich in 00 / FF records at random alignments, so that every offset within
  +-12 B of a 64-B ring-block boundary holds a 00 count, an FF count and an FF literal word
  start somewhere in the batch (checked: the ring carries 12 B between rounds,
  packed_kernels.hip decode_words_kernel);
- 00 FF chains (256 zero words per 2 bytes), with exact, short and 4-KiB slots.
Slots: the exact decoded size, 8 B short of it, a 4-KiB slot, or (for units that fail) a
random size. Checks: status, out_len (the required size on OUT_OF_SPACE), the bytes of OK units,
nothing written past out_len (OK) / out_cap (failed) or before the slot; a failed unit under
the two-pass decoder leaves its whole slot untouched.

Run under each forced mid-unit decoder (the `decoder` fixture) and under the default (AUTO) in a
batch of ~200K clean 4-KiB units, past the words decoder's routing threshold (a resident grid
of units over 1280 packed bytes), with the adversarial units scattered through it. Also: 64
expansion-heavy units in the headline batch cost at most 10% of its decode time (the words
decoder stops a lane at its slot's capacity, words_size_kernel finds the size)."""
import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
SENT = 0xA5
FRONT = 64  # canary bytes before each slot
BACK = 64   # canary bytes after each slot's capacity


def records(rng, target, p00=0.15, pff=0.15):
    """A valid packed stream of about `target` bytes: 00 c, FF w c + 8c literal, other tags."""
    out = bytearray()
    while len(out) < target:
        r = rng.random()
        if r < p00:
            c = int(rng.integers(0, 4)) if rng.random() < 0.85 else int(rng.integers(0, 256))
            out += bytes([0, c])
        elif r < p00 + pff:
            c = int(rng.integers(0, 4)) if rng.random() < 0.8 else int(rng.integers(0, 40))
            out += bytes([0xFF]) + rng.integers(0, 256, 8, dtype=np.uint8).tobytes() + bytes([c])
            out += rng.integers(0, 256, 8 * c, dtype=np.uint8).tobytes()
        else:
            t = int(rng.integers(1, 255))
            out += bytes([t]) + rng.integers(0, 256, bin(t).count("1"), dtype=np.uint8).tobytes()
    return bytes(out)


def record_starts(p):
    """(position, tag) of every record of a stream, as unpackPacked walks it (message.zig:101-141)."""
    i, n, out = 0, len(p), []
    while i < n:
        t = p[i]
        out.append((i, t))
        if t == 0:
            i += 2
        elif t == 0xFF:
            c = p[i + 9] if i + 9 < n else 0
            i += 10 + 8 * c
        else:
            i += 1 + bin(t).count("1")
    return out


def flip_one(rng, p):
    """Replace one tag or one 00 / FF count byte of a valid stream with a random byte."""
    starts = record_starts(p)
    pos, t = starts[int(rng.integers(0, len(starts)))]
    q = bytearray(p)
    if t == 0 and pos + 1 < len(q) and rng.random() < 0.5:
        pos += 1
    elif t == 0xFF and pos + 9 < len(q) and rng.random() < 0.5:
        pos += 9
    q[pos] = int(rng.integers(0, 256))
    return bytes(q)


def adversarial_units(seed, n_random=1200, n_flip=500, n_rich=700, n_chain=8):
    rng = np.random.default_rng(seed)
    units = []
    for _ in range(n_random):
        units.append(rng.integers(0, 256, int(rng.integers(513, 5121)), dtype=np.uint8).tobytes())
    for _ in range(n_flip):
        p = records(rng, int(rng.integers(600, 5000)), 0.05, 0.05)
        units.append(flip_one(rng, p)[:5120])
    for i in range(n_rich):
        p = records(rng, int(rng.integers(600, 5000)), 0.2, 0.2)
        if i % 7 == 3:
            p = p[:-int(rng.integers(1, 11))]  # cut: UNEXPECTED_EOF at the end
        units.append(p[:5120] if len(p) > 5120 else p)
    for i in range(n_chain):
        units.append(bytes([0, 0xFF]) * int(rng.integers(257, 700)))
    return [u if len(u) > 512 else u + bytes([0, 0]) * ((514 - len(u)) // 2 + 1) for u in units]


def expected(units):
    """Oracle status / decoded bytes per unit (message.zig:88-191)."""
    return [oracle.unpack(u) for u in units]


def choose_caps(rng, exp):
    caps = []
    for st, ref in exp:
        if st == oracle.OK:
            k = int(rng.integers(0, 4))
            size = len(ref)
            caps.append([size, max(size - 8, 0), 4096, size + 24][k] if size <= (1 << 16) else [4096, 8192][k & 1])
        else:
            caps.append(int(rng.integers(0, 16)) * 512)
    return caps


def layout(rng, units, caps, in_base=0, out_base=0):
    """Dense packed stream at random alignments; 8-B aligned slots with canaries around them."""
    n = len(units)
    in_off = np.zeros(n, dtype=np.int64)
    pos = in_base
    for i, u in enumerate(units):
        pos += int(rng.integers(0, 16))
        in_off[i] = pos
        pos += len(u)
    in_end = pos
    out_off = np.zeros(n, dtype=np.int64)
    o = out_base
    for i, c in enumerate(caps):
        o += FRONT + 8 * int(rng.integers(0, 16))  # slot starts at every 8-B phase of a 128-B line
        out_off[i] = o
        o += (c + 7) // 8 * 8 + BACK
    return in_off, in_end, out_off, o


def check(units, exp, caps, out, ooff, st, ol, strict):
    """strict: a failed unit leaves its whole slot untouched (the two-pass decoder)."""
    seen = set()
    for i, (ost, ref) in enumerate(exp):
        want = ost if ost != oracle.OK or len(ref) <= caps[i] else oracle.OUT_OF_SPACE
        seen.add(int(want))
        assert st[i] == want, (i, len(units[i]), int(st[i]), int(want))
        o, c = int(ooff[i]), caps[i]
        front = out[o - FRONT:o]
        assert (front == SENT).all(), (i, "bytes before the slot written")
        if want == oracle.OK:
            assert ol[i] == len(ref), (i, int(ol[i]), len(ref))
            assert out[o:o + len(ref)].tobytes() == ref, (i, "decoded bytes differ from the oracle")
            assert (out[o + len(ref):o + c + BACK] == SENT).all(), (i, "bytes past out_len written")
        else:
            if want == oracle.OUT_OF_SPACE:
                assert ol[i] == len(ref), (i, "required size", int(ol[i]), len(ref))
            else:
                assert ol[i] == 0, (i, int(ol[i]))
            lo = o if strict else o + c
            assert (out[lo:o + c + BACK] == SENT).all(), (i, int(want), "failed unit wrote where it may not")
    return seen


def run_batch(d_in, in_off, in_len, out_bytes, out_off, caps):
    d_out = torch.full((out_bytes,), SENT, dtype=torch.uint8, device=DEV)
    n = len(in_off)
    out_len = torch.full((n,), -1, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(DEV)
    cp.decode_batch(d_in, t(in_off), t(in_len), d_out, t(out_off), t(caps), out_len, status)
    torch.cuda.synchronize()
    return d_out, out_len.cpu().numpy(), status.cpu().numpy()


def boundary_coverage(units, in_off):
    """(kind, offset from the nearest 64-B aligned-space block boundary) pairs the batch holds."""
    cov = set()
    for u, off in zip(units, in_off):
        s = int(off) & 15
        for pos, t in record_starts(u):
            if t == 0:
                bs = [pos + 1]
                kinds = ["00 count"]
            elif t == 0xFF:
                bs = [pos + 9, pos + 10]
                kinds = ["FF count", "FF literal"]
            else:
                continue
            for b, kd in zip(bs, kinds):
                a = s + b
                d = (a + 32) % 64 - 32
                if -12 <= d <= 12:
                    cov.add((kd, d))
    return cov


def test_words_decoder_on_adversarial_mid_units(decoder):
    rng = np.random.default_rng(0xAD5E)
    units = adversarial_units(0xAD5E)
    exp = expected(units)
    caps = choose_caps(rng, exp)
    in_off, in_end, out_off, out_end = layout(rng, units, caps, 0, 0)
    cov = boundary_coverage(units, in_off)
    for kd in ("00 count", "FF count", "FF literal"):
        assert {d for k, d in cov if k == kd} == set(range(-12, 13)), kd
    buf = np.zeros(in_end, dtype=np.uint8)
    for u, o in zip(units, in_off):
        buf[o:o + len(u)] = np.frombuffer(u, dtype=np.uint8)
    d_in = torch.from_numpy(buf).to(DEV)
    d_out, ol, st = run_batch(d_in, in_off, [len(u) for u in units], out_end + BACK, out_off, caps)
    seen = check(units, exp, caps, d_out.cpu().numpy(), out_off, st, ol, strict=decoder == "twopass")
    assert seen == {oracle.OK, oracle.UNEXPECTED_EOF, oracle.OUT_OF_SPACE}


def test_auto_past_threshold_with_adversarial_units():
    """AUTO in a batch past the words decoder's threshold: ~220K clean 4-KiB units (p = 0.5, over
    1280 packed bytes, 4-KiB slots: the words decoder's share) with 2,400 adversarial units
    scattered through the batch order. Clean units round-trip; adversarial ones match the
    oracle, failed ones under the default contract (nothing past out_cap)."""
    if not cp.decoder_available("auto"):
        pytest.skip("no auto decoder")
    rng = np.random.default_rng(0xA070)
    nc, ub = 220_000, 4096
    d_clean = cp.generate(nc, ub, seed=0xC1EA, zero_thresh=128, device=torch.device(DEV))
    c_off, c_len = cp.uniform_layout(nc, ub, device=torch.device(DEV))
    slot = cp.encode_bound(ub)
    k_off, k_cap = cp.uniform_layout(nc, slot, device=torch.device(DEV))
    d_pk = torch.empty(nc * slot, dtype=torch.uint8, device=DEV)
    plen = torch.empty(nc, dtype=torch.int64, device=DEV)
    pst = torch.empty(nc, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_clean, c_off, c_len, d_pk, k_off, k_cap, plen, pst)
    torch.cuda.synchronize()
    assert int((pst != 0).sum()) == 0 and int((plen <= 1280).sum()) == 0

    units = adversarial_units(0xA071, n_random=1000, n_flip=500, n_rich=880, n_chain=20)
    exp = expected(units)
    caps = choose_caps(rng, exp)
    in_off, in_end, out_off, out_end = layout(rng, units, caps, nc * slot, nc * ub)
    buf = np.zeros(in_end - nc * slot, dtype=np.uint8)
    for u, o in zip(units, in_off):
        buf[o - nc * slot:o - nc * slot + len(u)] = np.frombuffer(u, dtype=np.uint8)
    d_in = torch.cat([d_pk, torch.from_numpy(buf).to(DEV)])

    na = len(units)
    n = nc + na
    order = rng.permutation(n)  # batch position of each entry: clean 0..nc-1, adversarial nc..
    all_in_off = np.concatenate([k_off.cpu().numpy(), in_off])[order]
    all_in_len = np.concatenate([plen.cpu().numpy(), np.array([len(u) for u in units], dtype=np.int64)])[order]
    all_out_off = np.concatenate([c_off.cpu().numpy(), out_off])[order]
    all_caps = np.concatenate([np.full(nc, ub, dtype=np.int64), np.array(caps, dtype=np.int64)])[order]
    with cp.decoder("auto"):
        d_out, ol, st = run_batch(d_in, all_in_off, all_in_len, out_end + BACK, all_out_off, all_caps)
    inv = np.empty(n, dtype=np.int64)
    inv[order] = np.arange(n)
    ci, ai = inv[:nc], inv[nc:]
    assert (st[ci] == 0).all() and (ol[ci] == ub).all()
    assert torch.equal(d_out[:nc * ub], d_clean), "clean units do not round-trip under AUTO"
    seen = check(units, exp, caps, d_out.cpu().numpy(), out_off, st[ai], ol[ai], strict=False)
    assert seen == {oracle.OK, oracle.UNEXPECTED_EOF, oracle.OUT_OF_SPACE}


def test_expansion_heavy_units_bounded_cost():
    """64 units of 00 FF chains (~2.5 KB packed, 256 zero words per record pair) in the 1M x 4 KiB
    headline batch: each reports OUT_OF_SPACE with its decoded size (oracle), and the batch decodes
    in at most 1.1x the clean batch's time (median of 7; the words decoder stops a lane at
    its 4-KiB slot, words_size_kernel walks the records)."""
    n, ub = 1 << 20, 4096
    dev = torch.device(DEV)
    d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=128, device=dev)
    in_off, in_len = cp.uniform_layout(n, ub, device=dev)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.empty(n, dtype=torch.int64, device=dev)
    pst = torch.empty(n, dtype=torch.int32, device=dev)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
    ulen = torch.empty(n, dtype=torch.int64, device=dev)
    ust = torch.empty(n, dtype=torch.int32, device=dev)

    def med_ms():
        ts = []
        s = torch.cuda.current_stream()
        for r in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
            e1.record(s)
            e1.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    clean = med_ms()
    assert bool(torch.equal(d_out, d_in))
    rng = np.random.default_rng(0xE4)
    heavy = np.sort(rng.choice(n, 64, replace=False))
    chain = bytes([0, 0xFF]) * 1250
    ref_size = oracle.decoded_size(chain)
    hb = torch.from_numpy(np.frombuffer(chain, dtype=np.uint8).copy()).to(DEV)
    for u in heavy.tolist():
        d_pk[u * slot:u * slot + len(chain)] = hb
        plen[u] = len(chain)
    torch.cuda.synchronize()
    with_heavy = med_ms()
    st = ust.cpu().numpy()
    ol = ulen.cpu().numpy()
    assert (st[heavy] == oracle.OUT_OF_SPACE).all() and (ol[heavy] == ref_size[1]).all()
    mask = np.ones(n, dtype=bool)
    mask[heavy] = False
    assert (st[mask] == 0).all()
    assert with_heavy <= 1.1 * clean, (with_heavy, clean)
