/*
 * packed_fast.c — a word-at-a-time CPU port of nullstyle/capnp-zig's packed codec, for
 * bench.py's cpu_baseline leg ONLY (not the checker, not the product).
 *
 * The checker (packed_oracle.c) restates message.zig:88-271 branch for branch and appends
 * output one byte at a time, which makes it a weak baseline (about 0.13 GiB/s per core for a
 * pack + unpack round trip). This file keeps the reference's algorithm and record choices
 * (message.zig:200-271 packPacked: zero runs, literal runs of words without a zero byte, tag +
 * nonzero bytes; message.zig:88-145 unpackPacked: the size pass of :152-191 first, then the
 * expansion) but does each step on whole words, as an optimised (ReleaseFast) build of the
 * reference would:
 *   - nonzero-byte masks by SWAR, a mixed word's bytes compacted with BMI2 pext and expanded
 *     with pdep, literal runs and zero runs by memcpy / memset;
 *   - pack's 8-byte stores may run up to 8 bytes past a record's end, so a unit needs that much
 *     slack; when the caller's capacity leaves less, or on any error (a size error, a truncated
 *     stream, a slot too small), the unit goes through the checker, whose result is then the
 *     answer by definition.
 * tests/test_fast_cpu.py compares it with the checker on every density, ragged and truncated
 * units and tight capacities.
 */
#include "packed_oracle.h"

#include <immintrin.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
static inline void st64(uint8_t* p, uint64_t v) { memcpy(p, &v, 8); }

/* 0x80 in every byte of v that is nonzero */
static inline uint64_t nonzero_hi(uint64_t v) {
    const uint64_t lo7 = 0x7F7F7F7F7F7F7F7FULL;
    return (((v & lo7) + lo7) | v) & 0x8080808080808080ULL;
}

/* message.zig:200-271, whole words; returns -1 when the unit needs the checker */
static int fast_pack_one(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    const size_t words = n / 8;
    if (n % 8 != 0 || cap < 9 * words + 1 + 8) return -1; /* size error or no slack: the checker */
    uint8_t* o = out;
    size_t i = 0;
    while (i < words) {
        const uint64_t x = ld64(in + 8 * i);
        if (x == 0) { /* zero run, <= 256 words */
            size_t r = 1;
            while (r < 256 && i + r < words && ld64(in + 8 * (i + r)) == 0) r++;
            o[0] = 0x00;
            o[1] = (uint8_t)(r - 1);
            o += 2;
            i += r;
            continue;
        }
        const uint64_t hi = nonzero_hi(x);
        if (hi == 0x8080808080808080ULL) { /* literal run of words without a zero byte, <= 256 */
            size_t r = 1;
            while (r < 256 && i + r < words && nonzero_hi(ld64(in + 8 * (i + r))) == 0x8080808080808080ULL) r++;
            o[0] = 0xFF;
            st64(o + 1, x);
            o[9] = (uint8_t)(r - 1);
            memcpy(o + 10, in + 8 * (i + 1), 8 * (r - 1));
            o += 10 + 8 * (r - 1);
            i += r;
            continue;
        }
        /* a mixed word: tag, then its nonzero bytes in byte order */
        const uint64_t mask = (hi >> 7) * 0xFF;
        const uint8_t tag = (uint8_t)_pext_u64(hi, 0x8080808080808080ULL);
        o[0] = tag;
        st64(o + 1, _pext_u64(x, mask));
        o += 1 + (size_t)__builtin_popcount(tag);
        i++;
    }
    *out_len = (size_t)(o - out);
    return 0;
}

/* message.zig:152-191 (the size pass), tags only; -1: an error the checker reports */
static int fast_size(const uint8_t* p, size_t n, size_t* total) {
    size_t t = 0, i = 0;
    while (i < n) {
        const uint8_t tag = p[i++];
        if (tag == 0x00) {
            if (i >= n) return -1;
            t += 8 * (1 + (size_t)p[i++]);
        } else if (tag == 0xFF) {
            if (i + 8 >= n) return -1;
            const size_t c = p[i + 8];
            i += 9;
            if (i + 8 * c > n) return -1;
            i += 8 * c;
            t += 8 * (1 + c);
        } else {
            i += (size_t)__builtin_popcount(tag);
            if (i > n) return -1;
            t += 8;
        }
    }
    *total = t;
    return 0;
}

/* message.zig:88-145: the size pass, then the expansion; -1 when the unit needs the checker */
static int fast_unpack_one(const uint8_t* p, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    size_t total = 0;
    if (fast_size(p, n, &total) != 0 || total > cap) return -1; /* errors and OUT_OF_SPACE: the checker */
    uint8_t* o = out;
    size_t i = 0;
    while (i < n) {
        const uint8_t tag = p[i++];
        if (tag == 0x00) {
            const size_t b = 8 * (1 + (size_t)p[i++]);
            memset(o, 0, b);
            o += b;
        } else if (tag == 0xFF) {
            const size_t c = p[i + 8];
            memcpy(o, p + i, 8);
            memcpy(o + 8, p + i + 9, 8 * c);
            o += 8 * (1 + c);
            i += 9 + 8 * c;
        } else {
            const uint64_t mask = _pdep_u64(tag, 0x0101010101010101ULL) * 0xFF;
            const size_t k = (size_t)__builtin_popcount(tag);
            uint64_t src;
            if (i + 8 <= n) {
                src = ld64(p + i);
            } else { /* the stream's last bytes: no read past the input */
                src = 0;
                memcpy(&src, p + i, k);
            }
            st64(o, _pdep_u64(src, mask));
            o += 8;
            i += k;
        }
    }
    *out_len = total;
    return 0;
}

void fast_pack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n, uint8_t* out, const uint64_t* out_off,
                     uint64_t* out_len, int32_t* status, int threads) {
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        size_t len = 0;
        const size_t m = in_off[i + 1] - in_off[i], cap = out_off[i + 1] - out_off[i];
        int st = fast_pack_one(in + in_off[i], m, out + out_off[i], cap, &len);
        if (st < 0) st = oracle_pack(in + in_off[i], m, out + out_off[i], cap, &len);
        out_len[i] = len;
        status[i] = st;
    }
    (void)threads;
}

void fast_unpack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n, uint8_t* out, const uint64_t* out_off,
                       uint64_t* out_len, int32_t* status, int threads) {
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        size_t len = 0;
        const size_t m = in_off[i + 1] - in_off[i], cap = out_off[i + 1] - out_off[i];
        int st = fast_unpack_one(in + in_off[i], m, out + out_off[i], cap, &len);
        if (st < 0) st = oracle_unpack(in + in_off[i], m, out + out_off[i], cap, &len);
        out_len[i] = len;
        status[i] = st;
    }
    (void)threads;
}
