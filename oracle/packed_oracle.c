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

/* appendSlice: one copy when the slice fits the capacity (literal runs, mixed words' bytes) */
static void sink_put_n(sink_t* s, const uint8_t* p, size_t n) {
    if (s->out && s->len + n <= s->cap) {
        memcpy(s->out + s->len, p, n);
        s->len += n;
        return;
    }
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

/* ------------------------------------------------------------------------
 * message.zig:699-969 Message.validate (and the helpers it calls, :11-18
 * decodeOffsetWords, :65-86 listContentBytes/Words, :279-285 decodeFarPointer,
 * :420-437 readWord/resolveFarLandingPad, :563-609 resolveInlineCompositeList,
 * message/bounds.zig:10-13 checkBounds), recursive as in the reference.
 * ------------------------------------------------------------------------ */
enum {
    V_OK = 0, V_EOS = 8, V_SEGCOUNT = 9, V_SEGLIMIT = 10, V_TRUNC = 13, V_EMPTY = 14, V_NEST = 15, V_SEGID = 16,
    V_PTR = 17, V_OOB = 18, V_TRAV = 19, V_FAR = 20, V_ICP = 21, V_LIST = 22
};

typedef struct {
    const uint8_t* data;
    uint32_t nseg;
    const uint64_t* off; /* segment byte offsets in data */
    const uint64_t* len; /* segment byte lengths */
    uint64_t remaining;
} vmsg_t;

static int64_t v_offset_words(uint64_t w) { /* :11-18 */
    uint32_t raw = (uint32_t)((w >> 2) & 0x3FFFFFFFu);
    return (raw & 0x20000000u) ? (int64_t)raw - ((int64_t)1 << 30) : (int64_t)raw;
}
static uint64_t v_word(const vmsg_t* m, uint32_t seg, uint64_t pos) { return load_le64(m->data + m->off[seg] + pos); }
static int v_bounds(const vmsg_t* m, uint32_t seg, uint64_t off, uint64_t size) { /* bounds.zig:10-13 */
    uint64_t end = off + size;
    if (end < off) return V_OOB;
    return end > m->len[seg] ? V_OOB : V_OK;
}
static int v_read(const vmsg_t* m, uint32_t seg, uint64_t pos, uint64_t* w) { /* :420-425 readWord */
    if (seg >= m->nseg) return V_SEGID;
    int e = v_bounds(m, seg, pos, 8);
    if (e) return e;
    *w = v_word(m, seg, pos);
    return V_OK;
}
static int v_consume(vmsg_t* m, uint64_t words) { /* :710-713 */
    if (words > m->remaining) return V_TRAV;
    m->remaining -= words;
    return V_OK;
}

static int v_pointer(vmsg_t* m, uint32_t seg, uint64_t pos, uint64_t word, uint64_t nesting);

/* pointers of `count` elements of (dw + pw) words at elements_offset (:855-866, :913-926, :956-967) */
static int v_elements(vmsg_t* m, uint32_t seg, uint64_t elements_offset, uint64_t count, uint64_t dw, uint64_t pw,
                      uint64_t nesting) {
    if (pw == 0 || count == 0) return V_OK;
    uint64_t stride = (dw + pw) * 8;
    for (uint64_t e = 0; e < count; ++e) {
        uint64_t ps = elements_offset + e * stride + dw * 8;
        for (uint64_t p = 0; p < pw; ++p) {
            uint64_t pp = ps + p * 8;
            int r = v_pointer(m, seg, pp, v_word(m, seg, pp), nesting);
            if (r) return r;
        }
    }
    return V_OK;
}

/* :929-968 validateInlineCompositeTag */
static int v_ic_tag(vmsg_t* m, uint32_t seg, uint64_t elements_offset, uint64_t tag, uint64_t nesting) {
    int64_t cs = v_offset_words(tag);
    if (cs < 0) return V_ICP;
    uint64_t count = (uint64_t)cs, dw = (tag >> 32) & 0xFFFF, pw = tag >> 48;
    uint64_t total_words = count * (dw + pw);
    if (total_words > UINT64_MAX / 8) return V_LIST; /* > maxInt(usize) / 8 (unreachable: < 2^46) */
    uint64_t total_bytes = total_words * 8;
    if (elements_offset > m->len[seg]) return V_OOB;
    if (total_bytes > m->len[seg] - elements_offset) return V_OOB;
    int r = v_consume(m, total_words);
    if (r) return r;
    return v_elements(m, seg, elements_offset, count, dw, pw, nesting);
}

/* :774-812 validateStructPointer */
static int v_struct(vmsg_t* m, uint32_t seg, uint64_t pos, uint64_t word, int has_ov, uint64_t ov, uint64_t nesting) {
    uint64_t ds = (word >> 32) & 0xFFFF, pc = word >> 48, so;
    if (has_ov) {
        so = ov;
    } else {
        int64_t s = (int64_t)pos + 8 + v_offset_words(word) * 8;
        if (s < 0) return V_OOB;
        so = (uint64_t)s;
    }
    uint64_t total_words = ds + pc, total_bytes = total_words * 8;
    if (so > m->len[seg]) return V_OOB;
    if (total_bytes > m->len[seg] - so) return V_OOB;
    int r = v_consume(m, total_words);
    if (r) return r;
    for (uint64_t i = 0; i < pc; ++i) {
        uint64_t pp = so + ds * 8 + i * 8;
        r = v_pointer(m, seg, pp, v_word(m, seg, pp), nesting);
        if (r) return r;
    }
    return V_OK;
}

static int v_list_bytes(uint64_t es, uint64_t count, uint64_t* bytes) { /* :65-79 */
    switch (es) {
        case 0: *bytes = 0; return V_OK;
        case 1: *bytes = (count + 7) / 8; return V_OK;
        case 2: *bytes = count; return V_OK;
        case 3: *bytes = count * 2; return V_OK;
        case 4: *bytes = count * 4; return V_OK;
        case 5: case 6: *bytes = count * 8; return V_OK;
        default: return V_PTR;
    }
}

/* :899-927 validateInlineCompositeList, with :563-609 resolveInlineCompositeList's list-pointer case
   (the only one validate reaches) */
static int v_ic_list(vmsg_t* m, uint32_t seg, uint64_t pos, uint64_t word, uint64_t nesting) {
    int64_t t = (int64_t)pos + 8 + v_offset_words(word) * 8;
    if (t < 0) return V_OOB;
    uint64_t tag_pos = (uint64_t)t, word_count = word >> 35, tag = 0;
    int r = v_read(m, seg, tag_pos, &tag);
    if (r) return r;
    if ((tag & 3) != 0) return V_ICP;
    int64_t cs = v_offset_words(tag);
    if (cs < 0) return V_ICP;
    uint64_t count = (uint64_t)cs, dw = (tag >> 32) & 0xFFFF, pw = tag >> 48;
    if (count * (dw + pw) > word_count) return V_ICP;
    uint64_t elements_offset = tag_pos + 8;
    r = v_bounds(m, seg, elements_offset, word_count * 8);
    if (r) return r;
    r = v_consume(m, word_count); /* :909 */
    if (r) return r;
    return v_elements(m, seg, elements_offset, count, dw, pw, nesting);
}

/* :814-897 validateListPointer */
static int v_list(vmsg_t* m, uint32_t seg, uint64_t pos, uint64_t word, int has_ov, uint64_t ov, uint64_t nesting) {
    uint64_t es = (word >> 32) & 7;
    if (es == 7 && !has_ov) return v_ic_list(m, seg, pos, word, nesting);
    if (es == 7) { /* layout B double-far inline composite (:827-869) */
        uint64_t word_count = word >> 35, tag_pos = ov, tag = 0;
        int r = v_read(m, seg, tag_pos, &tag);
        if (r) return r;
        if ((tag & 3) != 0) return V_ICP;
        int64_t cs = v_offset_words(tag);
        if (cs < 0) return V_ICP;
        uint64_t count = (uint64_t)cs, dw = (tag >> 32) & 0xFFFF, pw = tag >> 48;
        if (count * (dw + pw) > word_count) return V_ICP;
        uint64_t elements_offset = tag_pos + 8, total_bytes = word_count * 8;
        if (elements_offset > m->len[seg]) return V_OOB;
        if (total_bytes > m->len[seg] - elements_offset) return V_OOB;
        r = v_consume(m, word_count);
        if (r) return r;
        return v_elements(m, seg, elements_offset, count, dw, pw, nesting);
    }
    uint64_t count = word >> 35, co, bytes = 0;
    if (has_ov) {
        co = ov;
    } else {
        int64_t c = (int64_t)pos + 8 + v_offset_words(word) * 8;
        if (c < 0) return V_OOB;
        co = (uint64_t)c;
    }
    int r = v_list_bytes(es, count, &bytes);
    if (r) return r;
    if (co > m->len[seg]) return V_OOB;
    if (bytes > m->len[seg] - co) return V_OOB;
    r = v_consume(m, bytes ? (bytes + 7) / 8 : 0); /* listContentWords :81-86 */
    if (r) return r;
    if (es != 6 || count == 0) return V_OK;
    for (uint64_t i = 0; i < count; ++i) {
        uint64_t pp = co + 8 * i;
        r = v_pointer(m, seg, pp, v_word(m, seg, pp), nesting);
        if (r) return r;
    }
    return V_OK;
}

/* :736-772 validateFarPointer (with :430-437 resolveFarLandingPad) */
static int v_far(vmsg_t* m, uint64_t word, uint64_t nesting) {
    int dbl = (word >> 2) & 1;
    uint64_t pad_off = (word >> 3) & 0x1FFFFFFF;
    uint32_t fseg = (uint32_t)(word >> 32);
    if (fseg >= m->nseg) return V_SEGID;
    uint64_t landing = pad_off * 8;
    int r = v_bounds(m, fseg, landing, dbl ? 16 : 8);
    if (r) return r;
    uint64_t lw = 0, tw = 0;
    if (!dbl) {
        r = v_read(m, fseg, landing, &lw);
        if (r) return r;
        return v_pointer(m, fseg, landing, lw, nesting);
    }
    r = v_read(m, fseg, landing, &lw);
    if (r) return r;
    r = v_read(m, fseg, landing + 8, &tw);
    if (r) return r;
    if ((lw & 3) != 2) return V_FAR;
    if ((lw >> 2) & 1) return V_FAR;
    uint32_t lseg = (uint32_t)(lw >> 32);
    if (lseg >= m->nseg) return V_SEGID;
    uint64_t eo = ((lw >> 3) & 0x1FFFFFFF) * 8;
    if ((tw & 3) == 0) return v_ic_tag(m, lseg, eo, tw, nesting);
    if ((tw & 3) == 1) return v_list(m, lseg, 0, tw, 1, eo, nesting);
    return V_FAR;
}

/* :715-734 validatePointer */
static int v_pointer(vmsg_t* m, uint32_t seg, uint64_t pos, uint64_t word, uint64_t nesting) {
    if (word == 0) return V_OK;
    if (nesting == 0) return V_NEST;
    if (seg >= m->nseg) return V_SEGID;
    switch (word & 3) {
        case 0: return v_struct(m, seg, pos, word, 0, 0, nesting - 1);
        case 1: return v_list(m, seg, pos, word, 0, 0, nesting - 1);
        case 2: return v_far(m, word, nesting - 1);
        default: return V_PTR;
    }
}

int oracle_validate(const uint8_t* data, size_t n, uint64_t segment_count_limit, uint64_t traversal_limit_words,
                    uint64_t nesting_limit, uint64_t* words) {
    uint64_t off[512], len[512];
    uint32_t nseg = 0;
    *words = 0;
    int r = oracle_message_init(data, n, 512, off, len, &nseg);
    if (r == -1) return V_EOS;
    if (r == -2) return V_SEGCOUNT;
    if (r == -3) return V_SEGLIMIT;
    if (r) return V_TRUNC;
    /* :699-708 validate */
    if (nseg == 0) return V_EMPTY;
    if (nseg > segment_count_limit) return V_SEGLIMIT;
    if (len[0] < 8) return V_TRUNC;
    vmsg_t m = {data, nseg, off, len, traversal_limit_words};
    r = v_pointer(&m, 0, 0, v_word(&m, 0, 0), nesting_limit);
    if (r == V_OK) *words = traversal_limit_words - m.remaining;
    return r;
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

/* One connection's buffered bytes through readPackedMessage until no whole message is left, as
 * Connection.handleRead's loop does (level2/connection.zig:153-203 over reader.zig:84-156): the
 * CPU side of scripts/framer_crossover.py. Frames are written back to back into out; returns the
 * frames read, *used = bytes consumed, *out_total = frame bytes written. */
size_t oracle_read_stream(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* used,
                          size_t* out_total) {
    size_t pos = 0, o = 0, frames = 0;
    for (;;) {
        size_t len = 0, cons = 0;
        if (oracle_read_packed_message(in + pos, n - pos, out + o, cap - o, &len, &cons) != 0) break;
        pos += cons;
        o += len;
        ++frames;
    }
    *used = pos;
    *out_total = o;
    return frames;
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
