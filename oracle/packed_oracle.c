/*
 * packed_oracle.c — CPU restatement of nullstyle/capnp-zig's packed codec.
 *
 * TEST INFRASTRUCTURE ONLY (see packed_oracle.h). Each function follows the
 * reference function named in its comment, branch for branch, so that its
 * outputs and error classes are those of the Zig code. This file is the
 * checker the parity tests compare the HIP path against, and the CPU baseline
 * bench.py reports ("kind": "port"). It is never linked into the product.
 */
#include "packed_oracle.h"

#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum {
    ST_OK = 0,
    ST_INVALID_MESSAGE_SIZE = 1,
    ST_UNEXPECTED_EOF = 2,
    ST_OVERFLOW = 3,
    ST_OUT_OF_SPACE = 4,
    ST_INVALID_ARGUMENT = 5,
};

static uint64_t load_le64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

static uint32_t load_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* message.zig:196-198 */
int oracle_word_has_zero_byte(uint64_t v) {
    return ((v - 0x0101010101010101ULL) & ~v & 0x8080808080808080ULL) != 0;
}

/* Output sink with the semantics of std.ArrayList.append: count every byte,
 * store only while within capacity. */
typedef struct {
    uint8_t* out;
    size_t cap;
    size_t len;
} sink_t;

static void sink_put(sink_t* s, uint8_t b) {
    if (s->out && s->len < s->cap) s->out[s->len] = b;
    s->len++;
}

static void sink_put_n(sink_t* s, const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) sink_put(s, p[i]);
}

/* message.zig:200-271 packPacked */
int oracle_pack(const uint8_t* bytes, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    *out_len = 0;
    if (n % 8 != 0) return ST_INVALID_MESSAGE_SIZE; /* :201 */
    sink_t s = {out, out ? cap : 0, 0};
    size_t index = 0;
    while (index < n) { /* :207 */
        const uint8_t* word = bytes + index;
        uint64_t word_val = load_le64(word);
        if (word_val == 0) { /* :211-225 zero run, capped at 256 words */
            size_t run = 1;
            size_t scan = index + 8;
            while (run < 256 && scan + 8 <= n) {
                if (load_le64(bytes + scan) != 0) break;
                run++;
                scan += 8;
            }
            sink_put(&s, 0x00);
            sink_put(&s, (uint8_t)(run - 1));
            index += run * 8;
            continue;
        }
        if (!oracle_word_has_zero_byte(word_val)) { /* :231-251 literal run */
            size_t run = 1;
            size_t scan = index + 8;
            while (run < 256 && scan + 8 <= n) {
                if (oracle_word_has_zero_byte(load_le64(bytes + scan))) break;
                run++;
                scan += 8;
            }
            sink_put(&s, 0xFF);
            sink_put_n(&s, word, 8);
            sink_put(&s, (uint8_t)(run - 1));
            if (run > 1) sink_put_n(&s, bytes + index + 8, (run - 1) * 8);
            index += run * 8;
            continue;
        }
        /* :253-267 mixed word: tag + nonzero bytes in byte order */
        uint8_t tag = 0;
        uint8_t nonzero[8];
        size_t nonzero_len = 0;
        for (int i = 0; i < 8; ++i) {
            if (word[i] != 0) {
                tag |= (uint8_t)(1u << i);
                nonzero[nonzero_len++] = word[i];
            }
        }
        sink_put(&s, tag);
        sink_put_n(&s, nonzero, nonzero_len);
        index += 8;
    }
    *out_len = s.len;
    if (out && s.len > cap) return ST_OUT_OF_SPACE; /* out == NULL: size query */
    return ST_OK;
}

/* message.zig:152-191 estimateUnpackedSize */
int oracle_estimate_unpacked_size(const uint8_t* p, size_t n, size_t* out_size) {
    size_t total = 0;
    size_t index = 0;
    *out_size = 0;
    while (index < n) {
        uint8_t tag = p[index];
        index += 1;
        if (tag == 0x00) { /* :160-169 */
            if (total > SIZE_MAX - 8) return ST_OVERFLOW;
            total += 8;
            if (index >= n) return ST_UNEXPECTED_EOF;
            uint8_t count = p[index];
            index += 1;
            if (total > SIZE_MAX - (size_t)count * 8) return ST_OVERFLOW;
            total += (size_t)count * 8;
            continue;
        }
        if (tag == 0xFF) { /* :171-183 */
            if (index + 8 > n) return ST_UNEXPECTED_EOF;
            if (total > SIZE_MAX - 8) return ST_OVERFLOW;
            total += 8;
            index += 8;
            if (index >= n) return ST_UNEXPECTED_EOF;
            uint8_t count = p[index];
            index += 1;
            size_t byte_count = (size_t)count * 8;
            if (index + byte_count > n) return ST_UNEXPECTED_EOF;
            if (total > SIZE_MAX - byte_count) return ST_OVERFLOW;
            total += byte_count;
            index += byte_count;
            continue;
        }
        /* :186-189 regular tag */
        if (total > SIZE_MAX - 8) return ST_OVERFLOW;
        total += 8;
        size_t nonzero_bytes = (size_t)__builtin_popcount(tag);
        if (index + nonzero_bytes > n) return ST_UNEXPECTED_EOF;
        index += nonzero_bytes;
    }
    *out_size = total;
    return ST_OK;
}

/* message.zig:88-145 unpackPacked */
int oracle_unpack(const uint8_t* p, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    size_t total = 0;
    *out_len = 0;
    int st = oracle_estimate_unpacked_size(p, n, &total); /* :90 size pass first */
    if (st != ST_OK) return st;
    *out_len = total;
    if (total > cap || (!out && total > 0)) return ST_OUT_OF_SPACE;
    size_t o = 0;
    size_t index = 0;
    while (index < n) {
        uint8_t tag = p[index];
        index += 1;
        if (tag == 0x00) { /* :101-110 */
            uint8_t count = p[index];
            index += 1;
            size_t zero_bytes = (1 + (size_t)count) * 8;
            memset(out + o, 0, zero_bytes);
            o += zero_bytes;
            continue;
        }
        if (tag == 0xFF) { /* :112-128 */
            memcpy(out + o, p + index, 8);
            o += 8;
            index += 8;
            uint8_t count = p[index];
            index += 1;
            if (count > 0) {
                size_t byte_count = (size_t)count * 8;
                memcpy(out + o, p + index, byte_count);
                o += byte_count;
                index += byte_count;
            }
            continue;
        }
        /* :131-141 */
        memset(out + o, 0, 8);
        for (int bit = 0; bit < 8; ++bit) {
            if (tag & (1u << bit)) {
                out[o + bit] = p[index];
                index += 1;
            }
        }
        o += 8;
    }
    return ST_OK;
}

/* message.zig:341-394 Message.init (segment table parse only) */
int oracle_message_init(const uint8_t* data, size_t n, uint32_t max_segs,
                        uint64_t* seg_off, uint64_t* seg_len, uint32_t* seg_count) {
    *seg_count = 0;
    if (n < 4) return -1; /* readInt -> EndOfStream */
    uint32_t minus_one = load_le32(data);
    if (minus_one == 0xFFFFFFFFu) return -2; /* :346 InvalidSegmentCount */
    uint64_t count = (uint64_t)minus_one + 1;
    if (count > 512) return -3; /* :348 SegmentCountLimitExceeded */
    uint64_t padding_words = (count % 2 == 0) ? 1 : 0;
    uint64_t header_bytes = (1 + count + padding_words) * 4;
    if (header_bytes > n) return -4; /* :353 TruncatedMessage */
    uint64_t offset = header_bytes;
    for (uint64_t i = 0; i < count; ++i) {
        uint64_t size_words = load_le32(data + 4 + 4 * i);
        uint64_t end = offset + size_words * 8;
        if (end > n) return -4; /* :380 */
        if (i < max_segs) {
            seg_off[i] = offset;
            seg_len[i] = size_words * 8;
        }
        offset = end;
    }
    *seg_count = (uint32_t)count;
    return 0;
}

/* reader.zig:84-156 Reader.readPackedMessage */
int oracle_read_packed_message(const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                               size_t* out_len, size_t* consumed) {
    size_t r = 0;      /* read cursor */
    size_t len = 0;    /* out.items.len */
    int have_needed = 0;
    size_t needed = 0;
    *out_len = 0;
    *consumed = 0;
#define NEED_BYTE(var)                 \
    do {                               \
        if (r >= n) { *consumed = r; return -1; } \
        (var) = in[r++];               \
    } while (0)
#define EMIT(b)                                   \
    do {                                          \
        if (len >= cap) { *consumed = r; return -8; } \
        out[len++] = (uint8_t)(b);                \
    } while (0)
    for (;;) {
        if (have_needed && len >= needed) break; /* :91-93 */
        uint8_t tag;
        NEED_BYTE(tag);
        if (tag == 0x00) { /* :96-99 */
            uint8_t count;
            NEED_BYTE(count);
            size_t words = (size_t)count + 1;
            for (size_t i = 0; i < words * 8; ++i) EMIT(0);
        } else if (tag == 0xFF) { /* :100-111 */
            if (r + 8 > n) { *consumed = n; return -1; }
            for (int i = 0; i < 8; ++i) EMIT(in[r + i]);
            r += 8;
            uint8_t count;
            NEED_BYTE(count);
            if (count > 0) {
                size_t byte_count = (size_t)count * 8;
                if (r + byte_count > n) { *consumed = n; return -1; }
                for (size_t i = 0; i < byte_count; ++i) EMIT(in[r + i]);
                r += byte_count;
            }
        } else { /* :112-119 */
            uint8_t word[8] = {0};
            for (int i = 0; i < 8; ++i) {
                if (tag & (1u << i)) NEED_BYTE(word[i]);
            }
            for (int i = 0; i < 8; ++i) EMIT(word[i]);
        }
        if (!have_needed && len >= 4) { /* :121-144 */
            uint32_t minus_one = load_le32(out);
            if (minus_one == 0xFFFFFFFFu) { *consumed = r; return -2; }
            uint64_t count = (uint64_t)minus_one + 1;
            if (count > 512) { *consumed = r; return -3; }
            uint64_t padding_words = (count % 2 == 0) ? 1 : 0;
            uint64_t header_bytes = (1 + count + padding_words) * 4;
            if (len >= header_bytes) {
                uint64_t total_words = 0;
                for (uint64_t i = 0; i < count; ++i) total_words += load_le32(out + 4 + 4 * i);
                if (total_words > 8ull * 1024 * 1024) { *consumed = r; return -6; }
                needed = header_bytes + total_words * 8;
                have_needed = 1;
            }
        }
        if (have_needed && len >= needed) break; /* :146-148 */
    }
#undef NEED_BYTE
#undef EMIT
    *consumed = r;
    *out_len = len;
    if (len != needed) return -7; /* :151-153 InvalidPackedMessage */
    return 0;
}

void oracle_pack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n,
                       uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                       int32_t* status, int threads) {
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        size_t len = 0;
        size_t cap = out_off[i + 1] - out_off[i];
        int st = oracle_pack(in + in_off[i], in_off[i + 1] - in_off[i], out + out_off[i], cap, &len);
        out_len[i] = len;
        status[i] = st;
    }
    (void)threads;
}

void oracle_unpack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                         int32_t* status, int threads) {
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        size_t len = 0;
        size_t cap = out_off[i + 1] - out_off[i];
        int st = oracle_unpack(in + in_off[i], in_off[i + 1] - in_off[i], out + out_off[i], cap, &len);
        out_len[i] = len;
        status[i] = st;
    }
    (void)threads;
}

/* splitmix64 finaliser over (seed, unit, word); twin of the device generator. */
uint64_t oracle_mix64(uint64_t seed, uint64_t unit, uint64_t word) {
    uint64_t x = seed ^ (unit * 0x9E3779B97F4A7C15ULL) ^ (word * 0xC2B2AE3D27D4EB4FULL);
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

void oracle_generate(uint8_t* out, uint64_t n_units, uint64_t unit_bytes, uint64_t unit_base,
                     uint64_t seed, uint32_t zero_thresh, int threads) {
    uint64_t words = unit_bytes / 8;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n_units; ++i) {
        uint64_t u = unit_base + (uint64_t)i;
        uint8_t* dst = out + (uint64_t)i * unit_bytes;
        for (uint64_t w = 0; w < words; ++w) {
            uint64_t h = oracle_mix64(seed, u, w);
            uint64_t h2 = oracle_mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL, u, w);
            for (int k = 0; k < 8; ++k) {
                uint32_t r = (uint32_t)((h >> (8 * k)) & 0xFF);
                uint32_t v = (uint32_t)((h2 >> (8 * k)) & 0xFF);
                dst[w * 8 + k] = (r < zero_thresh) ? 0 : (uint8_t)(1 + v % 255);
            }
        }
    }
    (void)threads;
}
