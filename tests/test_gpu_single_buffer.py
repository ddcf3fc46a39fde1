"""Single-buffer host entry points on long buffers (message.zig:88-191, the Zig drop-in's
per-call path): capnp_packed_decode is one host-to-device copy and one device decode into
the caller's capacity, capnp_packed_decoded_size the size pass on the window-parallel
machinery for long units. Checked against the oracle (oracle/packed_oracle.c):
- buffers from 8 B to 16 MiB at p = 0.1 / 0.5 / 0.9: estimateUnpackedSize and
  unpackPacked bit-exact, also at an unaligned host address;
- OUT_OF_SPACE carries the required size and leaves the caller's buffer untouched;
- truncation (UnexpectedEof) from both entry points, no output written;
- an all-zero 16 MiB message (packed 1024x smaller: the 4x first guess is retried with the
  reported size);
- decoded_size_batch on a batch mixing long, serial-sized and mid units.
"""
import ctypes
import time

import numpy as np
import pytest

import capnp_packed as cp
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def message(nbytes, thr, seed=0xC0DE0B01):
    return oracle.generate(1, nbytes, seed=seed, zero_thresh=thr).tobytes()


def decode_raw(packed, cap, fill=0xAB):
    out = ctypes.create_string_buffer(bytes([fill]) * max(1, cap), max(1, cap))
    n = ctypes.c_size_t(7)
    st = cp.lib().capnp_packed_decode(packed, len(packed), out, cap, ctypes.byref(n))
    return st, n.value, out.raw[:cap]


@pytest.mark.parametrize("thr", [26, 128, 230])
def test_sizes_up_to_16_mib(thr):
    for nbytes in (8, 4096, 5128, 40960, 1 << 20, 16 << 20):
        data = message(nbytes, thr, seed=0xC0DE0B00 + nbytes)
        st, packed = oracle.pack(data)
        assert st == oracle.OK
        assert cp.estimate_unpacked_size(packed) == len(data) == oracle.decoded_size(packed)[1]
        assert cp.unpack_packed(packed) == data
        # the exact capacity in one call
        st, n, out = decode_raw(packed, len(data))
        assert (st, n) == (cp.OK, len(data)) and out == data


def test_16_mib_unaligned_host_and_timing():
    data = message(16 << 20, 128)
    _, packed = oracle.pack(data)
    buf = bytearray(len(packed) + 3)
    buf[3:] = packed
    src = (ctypes.c_char * len(buf)).from_buffer(buf)
    out = ctypes.create_string_buffer(len(data))
    n = ctypes.c_size_t()
    addr = ctypes.addressof(src) + 3
    assert cp.lib().capnp_packed_decode(ctypes.c_void_p(addr), len(packed), out, len(data), ctypes.byref(n)) == cp.OK
    assert n.value == len(data) and out.raw == data
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        cp.lib().capnp_packed_decode(ctypes.c_void_p(addr), len(packed), out, len(data), ctypes.byref(n))
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(f"16 MiB single-buffer unpack: {ms:.2f} ms (packed {len(packed)} B)")


def test_out_of_space_reports_size_and_writes_nothing():
    for nbytes in (64, 4096, 1 << 20, 16 << 20):
        data = message(nbytes, 128, seed=0xC0DE0B10 + nbytes)
        _, packed = oracle.pack(data)
        for cap in (0, len(data) - 8, len(data) // 2):
            st, n, out = decode_raw(packed, cap)
            assert st == cp.OUT_OF_SPACE and n == len(data)
            assert out == bytes([0xAB]) * cap


def test_truncation_is_unexpected_eof():
    for nbytes in (4096, 1 << 20, 16 << 20):
        data = message(nbytes, 26, seed=0xC0DE0B20 + nbytes)
        _, packed = oracle.pack(data)
        eofs = 0
        for cut in (1, 2, 5, 9, 10, 17, 100, 1001):
            p = packed[:-cut]
            exp, esize = oracle.decoded_size(p)
            st, n, out = decode_raw(p, len(data))
            if exp == oracle.UNEXPECTED_EOF:  # a cut can also land on a record boundary
                eofs += 1
                with pytest.raises(cp.UnexpectedEof):
                    cp.estimate_unpacked_size(p)
                assert (st, n) == (cp.UNEXPECTED_EOF, 0) and out == bytes([0xAB]) * len(data)
            else:
                assert cp.estimate_unpacked_size(p) == esize
                assert (st, n) == (cp.OK, esize) and out[:n] == oracle.unpack(p)[1]
        assert eofs >= 4


def test_all_zero_16_mib_retries_with_reported_size():
    data = bytes(16 << 20)
    _, packed = oracle.pack(data)
    assert len(packed) * 1000 < len(data)
    assert cp.estimate_unpacked_size(packed) == len(data)
    assert cp.unpack_packed(packed) == data
    st, n, _ = decode_raw(packed, 4 * len(packed))
    assert st == cp.OUT_OF_SPACE and n == len(data)


def test_decoded_size_batch_mixed_classes():
    rng = np.random.default_rng(11)
    sizes = [int(x) * 8 for x in rng.integers(0, 700, 300)]
    sizes[::37] = [int(x) * 8 for x in rng.integers(700, 200_000, len(sizes[::37]))]  # long: windows
    sizes[5] = 24 << 20  # one very long unit
    units, packed = [], []
    for i, nb in enumerate(sizes):
        d = message(nb, int(rng.choice([26, 128, 230])), seed=0xC0DE0B40 + i)
        _, p = oracle.pack(d)
        if i % 11 == 3 and len(p) > 2:
            p = p[:-int(rng.integers(1, min(len(p), 12)))]  # truncated
        units.append(d)
        packed.append(p)
    offs = np.zeros(len(packed), dtype=np.int64)
    pos = 0
    for i, p in enumerate(packed):
        pos += int(rng.integers(0, 16))  # unaligned packed starts
        offs[i] = pos
        pos += len(p)
    blob = np.zeros(pos + 16, dtype=np.uint8)
    for i, p in enumerate(packed):
        blob[offs[i]:offs[i] + len(p)] = np.frombuffer(p, dtype=np.uint8)
    d_in = torch.from_numpy(blob).cuda()
    in_off = torch.from_numpy(offs).cuda()
    in_len = torch.tensor([len(p) for p in packed], dtype=torch.int64, device="cuda")
    out_len = torch.full((len(packed),), -1, dtype=torch.int64, device="cuda")
    st = torch.full((len(packed),), -1, dtype=torch.int32, device="cuda")
    cp.decoded_size_batch(d_in, in_off, in_len, out_len, st)
    torch.cuda.synchronize()
    st, out_len = st.cpu().numpy(), out_len.cpu().numpy()
    for i, p in enumerate(packed):
        es, en = oracle.decoded_size(p)
        assert int(st[i]) == es, (i, len(p))
        assert int(out_len[i]) == (en if es == 0 else 0), (i, len(p))


def test_one_kernel_paths_around_their_limits():
    """Single-buffer decode up to 24 KiB of packed bytes and encode up to 4 KiB take one kernel
    (launch_decode_one / launch_encode_one); around both limits, at three
    densities, with truncations, a short capacity, a zero-heavy unit whose first 4x guess is too
    small, and an encode input that is not whole words: every result as the oracle's."""
    rng = np.random.default_rng(0x51)
    for thr in (26, 128, 230):
        for target in (24 * 1024 - 8, 24 * 1024, 24 * 1024 + 8):
            # grow the unpacked size until the packed size crosses the decode limit
            nbytes = 8 * int(target / 8 / {26: 1.03, 128: 0.63, 230: 0.24}[thr])
            data = message(nbytes, thr, seed=0xC0DE0B40 + thr + target)
            _, packed = oracle.pack(data)
            assert cp.unpack_packed(packed) == data, (thr, len(packed))
            st, n, out = decode_raw(packed, len(data))
            assert (st, n) == (cp.OK, len(data)) and out == data
            st, n, out = decode_raw(packed, len(data) - 8)
            assert (st, n) == (cp.OUT_OF_SPACE, len(data)) and out == bytes([0xAB]) * (len(data) - 8)
            p = packed[:-int(rng.integers(1, 12))]
            exp, esize = oracle.decoded_size(p)
            st, n, _ = decode_raw(p, len(data))
            assert st == (cp.UNEXPECTED_EOF if exp == oracle.UNEXPECTED_EOF else cp.OK)
    zeros = bytes(64 << 10)  # 2 packed bytes per 256 words: far past the 4x first guess
    _, pz = oracle.pack(zeros)
    assert len(pz) < 24 * 1024 and cp.unpack_packed(pz) == zeros
    for nbytes in (0, 8, 4088, 4096, 4104, 8192):
        data = message(nbytes, 128, seed=0xC0DE0B60 + nbytes) if nbytes else b""
        assert cp.pack_packed(data) == oracle.pack(data)[1], nbytes
    with pytest.raises(cp.InvalidMessageSize):
        cp.pack_packed(bytes(4092))
