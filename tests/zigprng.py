"""Restatement of Zig std's default PRNG, test infrastructure only.

The reference's fuzz tests (tests/serialization/message_test.zig:1057-1093) draw their
buffers from `std.Random.DefaultPrng.init(seed)` (Zig 0.15: `std.Random.Xoshiro256`,
xoshiro256++), through `random.uintLessThan(usize, 160)` and `random.bytes(buf)`. Zig is
not in this image, so this module restates the published algorithms:

- `Xoshiro256.init(s)` seeds its four state words with four SplitMix64 outputs of `s`
  (lib/std/Random/Xoshiro256.zig `seed`, lib/std/Random/SplitMix64.zig `next`);
- `next()` is xoshiro256++: rotl(s0 + s3, 23) + s0, then the xoshiro state update;
- `Random.bytes` is `Xoshiro256.fill`: one `next()` per 8 bytes, little-endian, and one more
  `next()` for a tail of 1-7 bytes (its low bytes);
- `Random.int(u64)` reads 8 bytes from `bytes`, i.e. one `next()`;
- `Random.uintLessThan(u64, n)` is Lemire's multiply-shift with the rejection threshold
  `(-n) mod n` (lib/std/Random.zig `uintLessThan`).

Pinned by Zig std's own known answer for this generator: `Xoshiro256.init(0)` yields
0x53175d61490b23df, 0x61da6f3dc380d507, 0x5c0fdf91ec9a7bfc, 0x02eebf8c3bbe5e1a,
0x7eca04ebaf4a5eea, 0x0543c37757f08d9a (the test "sequence" in
lib/std/Random/Xoshiro256.zig; std is not in this image, so the vector is quoted, not
read from a file: tests/test_zig_fuzz_corpus.py checks it). The corpus functions below
follow message_test.zig:1057-1093 line by line.
"""

M64 = (1 << 64) - 1

# message_test.zig:1058 and :1076
SEED_RAW = 0x3E22_7AB4_BD10_9C61    # "fuzz malformed buffers do not crash decode"
SEED_PACKED = 0xA7C4_1E59_F032_8D6B  # "fuzz malformed packed buffers do not crash decode"


def _splitmix64(state: int):
    state = (state + 0x9E3779B97F4A7C15) & M64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return state, z ^ (z >> 31)


def _rotl(x: int, k: int) -> int:
    return ((x << k) | (x >> (64 - k))) & M64


class Xoshiro256:
    """std.Random.Xoshiro256 (std.Random.DefaultPrng)."""

    def __init__(self, seed: int):
        st = seed & M64
        self.s = []
        for _ in range(4):
            st, v = _splitmix64(st)
            self.s.append(v)

    def next(self) -> int:
        s = self.s
        r = (_rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
        return r

    def bytes(self, n: int) -> bytes:
        """Random.bytes -> Xoshiro256.fill."""
        out = bytearray()
        for _ in range(n // 8):
            out += self.next().to_bytes(8, "little")
        if n % 8:
            out += self.next().to_bytes(8, "little")[: n % 8]
        return bytes(out)

    def uint_less_than(self, less_than: int) -> int:
        """Random.uintLessThan(u64, less_than)."""
        assert 0 < less_than <= M64
        x = self.next()
        m = x * less_than
        lo = m & M64
        if lo < less_than:
            t = (-less_than) & M64
            if t >= less_than:
                t -= less_than
                if t >= less_than:
                    t %= less_than
            while lo < t:
                x = self.next()
                m = x * less_than
                lo = m & M64
        return m >> 64


def fuzz_corpus(seed: int, count: int = 1024, max_len: int = 160):
    """The buffers of message_test.zig:1057-1073 / 1075-1093: `count` buffers, each of
    length uintLessThan(usize, 160), filled by random.bytes."""
    rng = Xoshiro256(seed)
    out = []
    for _ in range(count):
        n = rng.uint_less_than(max_len)
        out.append(rng.bytes(n))
    return out
