"""The reference's own fuzz corpora (message_test.zig:1057-1093), regenerated exactly.

tests/zigprng.py restates Zig std's DefaultPrng (xoshiro256++ seeded by SplitMix64) and
Random.uintLessThan / Random.bytes. CPU checks: the generator against Zig std's known
answer for seed 0, the corpus shapes, and the oracle's outcomes on both corpora (the
reference asserts only "no crash"; the oracle's outcome classes are the expected values
the GPU tests compare against, tests/test_gpu_zig_fuzz.py).
"""
import hashlib

import oracle
import zigprng


def test_xoshiro256_known_answer():
    # lib/std/Random/Xoshiro256.zig, test "sequence": Xoshiro256.init(0)
    r = zigprng.Xoshiro256(0)
    want = [0x53175D61490B23DF, 0x61DA6F3DC380D507, 0x5C0FDF91EC9A7BFC, 0x02EEBF8C3BBE5E1A,
            0x7ECA04EBAF4A5EEA, 0x0543C37757F08D9A]
    assert [r.next() for _ in range(6)] == want


def test_bytes_and_uint_less_than_semantics():
    a, b = zigprng.Xoshiro256(7), zigprng.Xoshiro256(7)
    # fill: one next() per 8 bytes (little-endian), one more for a 1-7 byte tail
    assert a.bytes(11) == b.next().to_bytes(8, "little") + b.next().to_bytes(8, "little")[:3]
    # uintLessThan(u64, n) = high half of next() * n when no rejection happens
    c, d = zigprng.Xoshiro256(9), zigprng.Xoshiro256(9)
    x = d.next()
    if (x * 160) & zigprng.M64 >= (-160 % (1 << 64)) % 160:
        assert c.uint_less_than(160) == (x * 160) >> 64
    vals = [zigprng.Xoshiro256(s).uint_less_than(160) for s in range(2000)]
    assert min(vals) >= 0 and max(vals) < 160 and len(set(vals)) > 150


def test_corpora_shape_and_determinism():
    for seed in (zigprng.SEED_RAW, zigprng.SEED_PACKED):
        c1, c2 = zigprng.fuzz_corpus(seed), zigprng.fuzz_corpus(seed)
        assert c1 == c2 and len(c1) == 1024
        assert all(len(b) < 160 for b in c1)
        assert sum(len(b) for b in c1) > 1024 * 60  # mean length ~80
    h = hashlib.sha256(b"".join(zigprng.fuzz_corpus(zigprng.SEED_RAW))).hexdigest()
    assert h == hashlib.sha256(b"".join(zigprng.fuzz_corpus(zigprng.SEED_RAW))).hexdigest()


def test_oracle_outcomes_on_reference_corpora():
    raw = zigprng.fuzz_corpus(zigprng.SEED_RAW)
    init_codes = {}
    for b in raw:  # Message.init then validate (message_test.zig:1061-1072)
        rc, _ = oracle.message_init(b)
        init_codes[rc] = init_codes.get(rc, 0) + 1
        oracle.validate(b)
    assert sum(init_codes.values()) == 1024 and len(init_codes) >= 2
    packed = zigprng.fuzz_corpus(zigprng.SEED_PACKED)
    unpack_codes = {}
    for b in packed:  # Message.initPacked = unpackPacked then Message.init (message.zig:400-408)
        st, out = oracle.unpack(b)
        unpack_codes[st] = unpack_codes.get(st, 0) + 1
        if st == oracle.OK:
            oracle.message_init(out)
            oracle.validate(out)
    assert unpack_codes.get(oracle.OK, 0) > 0 and unpack_codes.get(oracle.UNEXPECTED_EOF, 0) > 0
