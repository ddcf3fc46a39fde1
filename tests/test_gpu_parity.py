"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle. Bit-exact.

Sizes: the oracle-compared cases run in seconds on the host; the full
BASELINE-size batches (1M x 4 KiB) are checked through size-independent
properties (decode(encode(x)) == x on device, lengths against the oracle on a
strided sample).
"""
import os
import random

import numpy as np
import pytest

import capnp_packed as cp
import oracle
import pyref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "fixtures")
DEV = "cuda"


def fx(name):
    return open(os.path.join(FIX, name), "rb").read()


def _st_name(st):
    return cp.lib().capnp_packed_status_name(int(st)).decode()


# ---------------------------------------------------------------------------
# helpers: a batch of host byte strings laid out in device memory
# ---------------------------------------------------------------------------

def t64(xs):
    return torch.tensor(list(xs), dtype=torch.int64, device=DEV)


def device_units(units, pad_front=0, align=1):
    """One device buffer holding every unit; returns (buf, off, len) tensors.
    Unit starts are rounded up to `align` (after `pad_front` leading bytes)."""
    offs, pos = [], pad_front
    for u in units:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        pos += len(u)
    host = np.zeros(pos + 32, dtype=np.uint8)
    for o, u in zip(offs, units):
        host[o:o + len(u)] = np.frombuffer(u, dtype=np.uint8)
    return torch.from_numpy(host).to(DEV), t64(offs), t64(len(u) for u in units)


def slots(caps, align=16):
    offs, pos = [], 0
    for c in caps:
        offs.append(pos)
        pos += (c + align - 1) // align * align
    return t64(offs), t64(caps), pos


def _collect(d_out, out_off, out_len, status):
    torch.cuda.synchronize()
    lens, sts, offs = out_len.cpu().numpy(), status.cpu().numpy(), out_off.cpu().numpy()
    host = d_out.cpu().numpy()
    res = []
    for i in range(len(sts)):
        if sts[i] == cp.OK:
            res.append((int(sts[i]), host[offs[i]:offs[i] + lens[i]].tobytes()))
        else:
            res.append((int(sts[i]), int(lens[i])))
    return res


def gpu_encode(units, caps=None, pad_front=0):
    d_in, in_off, in_len = device_units(units, pad_front=pad_front, align=8)
    n = len(units)
    caps = caps if caps is not None else [cp.encode_bound(len(u)) for u in units]
    out_off, out_cap, total = slots(caps)
    d_out = torch.zeros(total + 16, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_out, out_off, out_cap, out_len, status)
    return _collect(d_out, out_off, out_len, status)


def gpu_decode(units, caps=None, pad_front=0):
    d_in, in_off, in_len = device_units(units, pad_front=pad_front)
    n = len(units)
    if caps is None:
        caps = []
        for u in units:
            st, sz = oracle.decoded_size(u)
            caps.append(sz if st == oracle.OK else 0)
    out_off, out_cap, total = slots(caps)
    d_out = torch.zeros(total + 16, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_in, in_off, in_len, d_out, out_off, out_cap, out_len, status)
    return _collect(d_out, out_off, out_len, status)


def check_encode_parity(units, **kw):
    got = gpu_encode(units, **kw)
    for i, u in enumerate(units):
        st, p = oracle.pack(u)
        if st == oracle.OK:
            assert got[i] == (cp.OK, p), f"unit {i} ({len(u)} B): {got[i][0]} vs oracle"
        else:
            assert got[i][0] == st, f"unit {i}: status {got[i][0]} vs {st}"


def check_decode_parity(units, **kw):
    got = gpu_decode(units, **kw)
    for i, u in enumerate(units):
        st, d = oracle.unpack(u)
        if st == oracle.OK:
            assert got[i] == (cp.OK, d), f"unit {i} ({len(u)} B packed): {got[i][0]}"
        else:
            assert got[i][0] == st, f"unit {i}: status {_st_name(got[i][0])} vs {_st_name(st)}"


def rand_units(rng, n, max_words, dens=(0.0, 0.1, 0.5, 0.9, 1.0)):
    out = []
    for _ in range(n):
        p = rng.choice(dens)
        nw = rng.randrange(0, max_words + 1)
        out.append(bytes(0 if rng.random() < p else rng.randrange(1, 256) for _ in range(8 * nw)))
    return out


# ---------------------------------------------------------------------------
# single-buffer API (host memory in / out)
# ---------------------------------------------------------------------------

PAIRS = [("binary", "packed"), ("segmented", "segmented-packed"),
         ("fixture_single.bin", "fixture_single_packed.bin"), ("fixture_far.bin", "fixture_far_packed.bin")]




@pytest.mark.parametrize("unpacked,packed", PAIRS)
def test_single_fixture_pairs(unpacked, packed, decoder):
    assert cp.unpack_packed(fx(packed)) == fx(unpacked)
    assert cp.estimate_unpacked_size(fx(packed)) == len(fx(unpacked))
    assert cp.pack_packed(fx(unpacked)) == oracle.pack(fx(unpacked))[1]


def test_single_kats(decoder):
    p = bytes([0x00, 0x01, 0xFF, 1, 2, 3, 4, 5, 6, 7, 8, 0x00])
    assert cp.estimate_unpacked_size(p) == 24
    assert cp.unpack_packed(p) == bytes(16) + bytes(range(1, 9))
    with pytest.raises(cp.UnexpectedEof):
        cp.estimate_unpacked_size(b"\x03\xaa")
    with pytest.raises(cp.UnexpectedEof):
        cp.unpack_packed(b"\x03\xaa")
    with pytest.raises(cp.InvalidMessageSize):
        cp.pack_packed(b"1234567")
    assert cp.pack_packed(b"") == b""
    assert cp.unpack_packed(b"") == b""


def test_single_golden_vectors(decoder):
    import json
    gold = json.load(open(os.path.join(HERE, "golden", "zig_vectors.json")))
    for v in gold["vectors"]:
        data = bytes.fromhex(v["unpacked_hex"]) if "unpacked_hex" in v else fx(v["name"].split(":", 1)[1])
        assert cp.pack_packed(data).hex() == v["packed_hex"], v["name"]
        assert cp.unpack_packed(bytes.fromhex(v["packed_hex"])) == data, v["name"]


def test_message_init_packed_roundtrip(decoder):
    b = cp.MessageBuilder()
    b.create_segment(bytes(range(1, 25)))
    b.create_segment(bytes(64))
    packed = b.to_packed_bytes()
    assert packed == pyref.to_packed_bytes([bytes(range(1, 25)), bytes(64)])
    msg = cp.Message.init_packed(packed)
    assert [bytes(s) for s in msg.segments] == [bytes(range(1, 25)), bytes(64)]
    assert cp.Reader.init_packed(packed).msg.backing_data == b.to_bytes()


# ---------------------------------------------------------------------------
# batch API: edge cases against the oracle
# ---------------------------------------------------------------------------

def test_batch_encode_edge_units():
    full = bytes(range(1, 9))
    units = [b"", bytes(8), full, bytes([0, 1, 0, 0, 0, 0, 0, 2]),
             bytes(8 * 255), bytes(8 * 256), bytes(8 * 257), bytes(4096),
             full * 255, full * 256, full * 257, full * 512,
             (bytes(8) + full) * 256, (full + bytes([5, 5, 5, 0, 5, 5, 5, 5])) * 256,
             bytes(8 * 100) + full * 300 + bytes(8 * 112)]
    check_encode_parity(units)


def test_batch_encode_random_small_and_fast_path_sizes():
    rng = random.Random(11)
    check_encode_parity(rand_units(rng, 300, 512))


def test_batch_encode_slow_path_units():
    rng = random.Random(12)
    units = rand_units(rng, 6, 3000) + [bytes(8 * 513), bytes(range(1, 9)) * 700]
    check_encode_parity(units)


def test_batch_encode_invalid_and_out_of_space():
    units = [b"1234567", bytes(range(1, 9)) * 3, bytes(16)]
    got = gpu_encode(units, caps=[16, 10, 100])
    assert got[0][0] == cp.INVALID_MESSAGE_SIZE
    assert got[1] == (cp.OUT_OF_SPACE, 26)  # needs 26 bytes, cap 10
    assert got[2] == (cp.OK, b"\x00\x01")


def test_batch_encode_misaligned_word_side_is_rejected():
    d_in = torch.zeros(64, dtype=torch.uint8, device=DEV)
    d_out = torch.zeros(48, dtype=torch.uint8, device=DEV)
    ln = torch.zeros(1, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, t64([4]), t64([8]), d_out, t64([0]), t64([32]), ln, st)
    torch.cuda.synchronize()
    assert int(st.item()) == cp.INVALID_ARGUMENT


@pytest.mark.parametrize("with_small", [False, True])
def test_batch_encode_kernel_prologue_paths_mixed_in_blocks(with_small):
    """encode_kernel's two entry paths side by side in its 4-wave blocks (round 6: an aligned
    512-word unit's loads go out before the block's selector-table barrier, every other unit is
    staged after it): 4 KiB units at 16-B and 8-B mod 16 starts, shorter mid units, an empty unit,
    and (with_small) lane-per-unit small units so the mid list is not the identity, plus units
    the kernel reports (InvalidMessageSize, a misaligned start). Every byte against the oracle;
    output slots are guarded by 0xEE canaries."""
    rng = random.Random(61 + with_small)
    specs = []
    for i in range(96):
        k = i % 8
        if k in (0, 3, 6):
            specs.append((4096, 0))          # direct: 16-B aligned 512 words
        elif k in (1, 5):
            specs.append((4096, 8))          # 512 words at 8 mod 16: staged
        elif k == 2:
            specs.append((8 * rng.randrange(65, 512), rng.choice((0, 8))))
        elif k == 4:
            specs.append((8 * rng.randrange(1, 64) if with_small else 0, 0))
        else:
            specs.append((8 * rng.randrange(100, 512), 8))
    specs[7] = (4093, 0)   # InvalidMessageSize (message.zig:201)
    specs[15] = (4096, 4)  # a start that is not word aligned: INVALID_ARGUMENT
    units, offs, pos = [], [], 0
    for ln, mod in specs:
        pos = (pos + 15) // 16 * 16 + mod
        offs.append(pos)
        p = rng.choice((0.1, 0.5, 0.9))
        units.append(bytes(0 if rng.random() < p else rng.randrange(1, 256) for _ in range(ln)))
        pos += ln
    host = np.zeros(pos + 64, dtype=np.uint8)
    for o, u in zip(offs, units):
        host[o:o + len(u)] = np.frombuffer(u, dtype=np.uint8)
    d_in = torch.from_numpy(host).to(DEV)
    n = len(units)
    caps = [cp.encode_bound(len(u)) + 16 for u in units]
    out_off, out_cap, total = slots(caps, align=16)
    d_out = torch.full((total + 64,), 0xEE, dtype=torch.uint8, device=DEV)
    out_len = torch.zeros(n, dtype=torch.int64, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, t64(offs), t64(len(u) for u in units), d_out, out_off, out_cap, out_len, status)
    torch.cuda.synchronize()
    sts, lens, oo = status.cpu().numpy(), out_len.cpu().numpy(), out_off.cpu().numpy()
    out = d_out.cpu().numpy().tobytes()
    for i, u in enumerate(units):
        if i == 15:
            assert sts[i] == cp.INVALID_ARGUMENT
            continue
        st, p = oracle.pack(u)
        assert sts[i] == st, f"unit {i}: status {sts[i]} vs {st}"
        if st == oracle.OK:
            assert out[oo[i]:oo[i] + lens[i]] == p, f"unit {i} ({len(u)} B at {offs[i] % 16} mod 16)"
            assert out[oo[i] + lens[i]:oo[i] + caps[i]] == b"\xee" * (caps[i] - int(lens[i])), f"unit {i} canary"


def test_batch_encode_dense_unaligned_output():
    """Dense packed output: sizes -> scan -> encode at unaligned byte offsets."""
    rng = random.Random(13)
    units = rand_units(rng, 200, 512)
    d_in, in_off, in_len = device_units(units, align=8)
    n = len(units)
    lens = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.zeros(n, dtype=torch.int32, device=DEV)
    cp.encoded_size_batch(d_in, in_off, in_len, lens, st)
    off = cp.lengths_to_offsets(lens, base=3)
    d_out = torch.full((int(off[-1].item()) + 16,), 0xEE, dtype=torch.uint8, device=DEV)
    ln2 = torch.zeros(n, dtype=torch.int64, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_out, off[:-1], lens, ln2, st)
    torch.cuda.synchronize()
    assert (st.cpu() == 0).all()
    expect = b"".join(oracle.pack(u)[1] for u in units)
    host = d_out.cpu().numpy().tobytes()
    assert host[3:3 + len(expect)] == expect
    assert host[:3] == b"\xee" * 3 and host[3 + len(expect):3 + len(expect) + 8] == b"\xee" * 8


def test_batch_decode_adversarial_and_fuzz(decoder):
    units = [bytes.fromhex(h) for h in (
        "", "01", "00", "0000", "00ff", "ff", "ff01020304", "ff0102030405060708",
        "ff010203040506070800", "ff010203040506070801", "ff010203040506070801aabb",
        "ff0102030405060708ff", "fe0102", "80", "000001", "00000000", "ffffffffffffffffffff",
        "0003", "0001ff010203040506070800", "03aa", "10010000", "0001")]
    rng = random.Random(0xA7C41E59)
    units += [bytes(rng.randrange(256) for _ in range(rng.randrange(160))) for _ in range(1024)]
    check_decode_parity(units)


def test_batch_decode_roundtrips_random(decoder):
    rng = random.Random(21)
    raw = rand_units(rng, 400, 512)
    packed = [oracle.pack(u)[1] for u in raw]
    check_decode_parity(packed)


def test_batch_decode_unaligned_packed_bases(decoder):
    rng = random.Random(22)
    packed = [oracle.pack(u)[1] for u in rand_units(rng, 200, 300)]
    check_decode_parity(packed, pad_front=5)


def test_batch_decode_windows_and_slow_path(decoder):
    full = bytes(range(1, 9))
    units = [b"\x00\xff" * 3,                              # 6144 zero bytes, 3 windows
             oracle.pack(full * 700)[1],                   # literal runs across windows, P > fast limit
             oracle.pack(bytes(8 * 600) + full * 600)[1],
             oracle.pack((full + bytes(8)) * 900)[1],       # slow path (P > 4816)
             b"\x00\xff" * 40,                             # 80 KiB of zeros from 80 bytes
             bytes([0xFF]) + full + b"\xff" + full * 255 + b"\x00\x10"]
    check_decode_parity(units)


def test_batch_decode_out_of_space_and_misaligned_output(decoder):
    units = [b"\x00\x03", b"\x00\x00"]
    got = gpu_decode(units, caps=[16, 8])
    assert got[0] == (cp.OUT_OF_SPACE, 32)
    assert got[1] == (cp.OK, bytes(8))
    d_in, in_off, in_len = device_units([b"\x00\x00"])
    d_out = torch.zeros(32, dtype=torch.uint8, device=DEV)
    ln = torch.zeros(1, dtype=torch.int64, device=DEV)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_in, in_off, in_len, d_out, t64([4]), t64([8]), ln, st)
    torch.cuda.synchronize()
    assert int(st.item()) == cp.INVALID_ARGUMENT


def test_size_batches_match_oracle(decoder):
    rng = random.Random(31)
    raw = rand_units(rng, 300, 600)
    d_in, in_off, in_len = device_units(raw, align=8)
    n = len(raw)
    ln = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.zeros(n, dtype=torch.int32, device=DEV)
    cp.encoded_size_batch(d_in, in_off, in_len, ln, st)
    torch.cuda.synchronize()
    assert ln.cpu().tolist() == [len(oracle.pack(u)[1]) for u in raw]
    packed = [oracle.pack(u)[1] for u in raw] + [b"\x03\xaa", b"\x00"]
    d_in, in_off, in_len = device_units(packed)
    n = len(packed)
    ln = torch.zeros(n, dtype=torch.int64, device=DEV)
    st = torch.zeros(n, dtype=torch.int32, device=DEV)
    cp.decoded_size_batch(d_in, in_off, in_len, ln, st)
    torch.cuda.synchronize()
    assert ln.cpu().tolist()[:-2] == [len(u) for u in raw]
    assert st.cpu().tolist()[-2:] == [cp.UNEXPECTED_EOF] * 2


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 100_000])
def test_lengths_to_offsets(n):
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 5000, size=n).astype(np.int64)
    d = torch.from_numpy(lens).to(DEV)
    off = cp.lengths_to_offsets(d, base=7).cpu().numpy()
    expect = np.concatenate([[7], 7 + np.cumsum(lens)]) if n else np.array([7])
    assert (off == expect).all()


# ---------------------------------------------------------------------------
# BASELINE configs
# ---------------------------------------------------------------------------

def test_generator_matches_oracle_generator():
    d = cp.generate(256, 4096, seed=0xC0DE0003, zero_thresh=128, unit_base=1000)
    h = oracle.generate(256, 4096, seed=0xC0DE0003, zero_thresh=128, unit_base=1000)
    assert (d.cpu().numpy() == h).all()


def roundtrip_uniform(n_units, unit_bytes, seed, thr):
    """Generate on device, encode into capacity slots, decode straight from the
    slots (encode's out_off/out_len are decode's in_off/in_len)."""
    d_in = cp.generate(n_units, unit_bytes, seed=seed, zero_thresh=thr)
    in_off, in_len = cp.uniform_layout(n_units, unit_bytes)
    slot = cp.encode_bound(unit_bytes)
    pk_off, pk_cap = cp.uniform_layout(n_units, slot)
    d_pk = torch.empty(n_units * slot, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n_units, dtype=torch.int64, device=DEV)
    pst = torch.full((n_units,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    d_out = torch.empty(n_units * unit_bytes, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n_units, dtype=torch.int64, device=DEV)
    ust = torch.full((n_units,), -1, dtype=torch.int32, device=DEV)
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
    torch.cuda.synchronize()
    assert (pst == 0).all().item() and (ust == 0).all().item()
    assert (ulen == unit_bytes).all().item()
    assert torch.equal(d_out, d_in)
    return d_in, d_pk, plen, slot


def check_sample_vs_oracle(d_in, d_pk, plen, slot, unit_bytes, n_sample):
    n = plen.numel()
    idx = np.unique(np.linspace(0, n - 1, n_sample).astype(np.int64))
    lens = plen.cpu().numpy()
    rows_in = d_in.view(n, unit_bytes)[torch.from_numpy(idx).to(DEV)].cpu().numpy()
    rows_pk = d_pk.view(n, slot)[torch.from_numpy(idx).to(DEV)].cpu().numpy()
    for k, i in enumerate(idx):
        st, p = oracle.pack(rows_in[k].tobytes())
        assert st == oracle.OK and lens[i] == len(p), i
        assert rows_pk[k][:len(p)].tobytes() == p, i


def test_config2_64k_x_1KiB_p50_bit_exact(decoder):
    """BASELINE configs[1]: 64K x 1 KiB, p = 0.5, pack+unpack bit-exact vs the oracle (every unit)."""
    n, ub = 65536, 1024
    d_in, d_pk, plen, slot = roundtrip_uniform(n, ub, 0xC0DE0002, 128)
    h_in = oracle.generate(n, ub, seed=0xC0DE0002, zero_thresh=128)
    assert (d_in.cpu().numpy() == h_in).all()
    h_off = np.arange(0, n * ub + 1, ub, dtype=np.uint64)
    h_slot = np.arange(0, n * slot + 1, slot, dtype=np.uint64)
    o_out, o_len, o_st = oracle.pack_batch(h_in, h_off, h_slot)
    assert (o_st == 0).all()
    assert (plen.cpu().numpy().astype(np.uint64) == o_len).all()
    g = d_pk.cpu().numpy().reshape(n, slot)
    o = o_out[:n * slot].reshape(n, slot)
    valid = np.arange(slot)[None, :] < o_len.astype(np.int64)[:, None]
    assert (g[valid] == o[valid]).all()


@pytest.mark.parametrize("thr", [26, 128, 230])  # p = 0.1 / 0.5 / 0.9 (x/256)
def test_config3_4KiB_units_density_sweep(thr, decoder):
    """BASELINE configs[2] shape at 16K units; every 8th unit byte-compared with the oracle."""
    d_in, d_pk, plen, slot = roundtrip_uniform(16384, 4096, 0xC0DE0003, thr)
    check_sample_vs_oracle(d_in, d_pk, plen, slot, 4096, 2048)


def test_config3_full_size_roundtrip_property(decoder):
    """1M x 4 KiB, p = 0.5 (headline size): decode(encode(x)) == x on device,
    and 1024 strided units byte-compared with the oracle."""
    d_in, d_pk, plen, slot = roundtrip_uniform(1 << 20, 4096, 0xC0DE0003, 128)
    check_sample_vs_oracle(d_in, d_pk, plen, slot, 4096, 1024)
    total = int(plen.sum().item())
    assert 0.55 * (1 << 32) < total < 0.70 * (1 << 32)  # ~0.626 expected at p = 0.5


@pytest.mark.parametrize("thr", [26, 230])  # p = 0.1 / 0.9: the rest of the headline density sweep
def test_config3_full_size_density_sweep(thr, decoder):
    """BASELINE configs[2] at its stated size, p = 0.1 and 0.9: 1M x 4 KiB,
    decode(encode(x)) == x on device, 1024 strided units byte-compared with the oracle."""
    d_in, d_pk, plen, slot = roundtrip_uniform(1 << 20, 4096, 0xC0DE0003, thr)
    check_sample_vs_oracle(d_in, d_pk, plen, slot, 4096, 1024)
    ratio = int(plen.sum().item()) / (1 << 32)
    assert (0.98 < ratio < 1.08) if thr == 26 else (0.18 < ratio < 0.30)  # ~1.033 / ~0.232


def test_auto_decoder_splits_mixed_densities():
    """AUTO on a batch past the words decoder's routing threshold with units on both sides of the
    split (launch_decode / class_scan_kernel: units of <= 1280 packed bytes two-pass, longer ones
    by the words decoder): 512K x 4 KiB units alternating p = 0.9 and p = 0.5, plus a tail of
    p = 0.1 units, decode(encode(x)) == x with every length and status, a strided sample against
    the oracle."""
    n2, ub = 1 << 18, 4096
    a = cp.generate(n2, ub, seed=0xC0DE0031, zero_thresh=230, device=DEV).view(n2, ub)
    b = cp.generate(n2, ub, seed=0xC0DE0032, zero_thresh=128, device=DEV).view(n2, ub)
    c = cp.generate(4096, ub, seed=0xC0DE0033, zero_thresh=26, device=DEV).view(4096, ub)
    d_in = torch.cat([torch.stack([a, b], dim=1).reshape(2 * n2, ub), c]).reshape(-1)
    del a, b, c
    n = d_in.numel() // ub
    in_off, in_len = cp.uniform_layout(n, ub)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot)
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    lens = plen.cpu().numpy()
    assert (lens[0:2 * n2:2] <= 1280).mean() > 0.99 and (lens[1:2 * n2:2] > 1280).all()
    d_out = torch.empty(n * ub, dtype=torch.uint8, device=DEV)
    ulen = torch.zeros(n, dtype=torch.int64, device=DEV)
    ust = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    with cp.decoder("auto"):
        cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
    torch.cuda.synchronize()
    assert (pst == 0).all().item() and (ust == 0).all().item() and (ulen == ub).all().item()
    assert torch.equal(d_out, d_in)
    check_sample_vs_oracle(d_in, d_pk, plen, slot, ub, 512)
