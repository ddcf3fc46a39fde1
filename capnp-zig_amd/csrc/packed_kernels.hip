// packed_kernels.hip — CDNA4 (gfx950) kernels for the Cap'n Proto packed codec.
//
// Reference semantics (Zig rules, NOT canonical C++ capnp):
//   encode  nullstyle/capnp-zig src/serialization/message.zig:200-271 (packPacked)
//   decode  message.zig:88-145 (unpackPacked) with the size pass of :152-191
//
// Execution model. No MFMA: this is byte compaction, HBM-bound.
// Every batch is first split into size classes (class_count / class_scan /
// class_scatter): small units (lane per unit), mid units (wave per unit)
// and long units (> one 512-word tile / > 5 KiB packed), which run on a side stream of
// the caller's stream, beside the main grid.
//   encode  small: encode_stream_kernel, lane per unit. Mid: one 64-lane wave per unit of
//           <= 512 words (encode_kernel): the unit is staged in the wave's LDS slice
//           with coalesced 16-B loads; lane j owns words [8j, 8j+8); zero-byte tags come
//           from SWAR + a multiply gather; greedy 256-capped zero / literal runs are
//           resolved with wave max/min scans of break positions; a wave sum scan gives
//           each lane its output offset; lanes OR their records into an LDS byte stream
//           written back with coalesced stores. Long: tile-parallel (long_tiles_kernel,
//           tile_encode_kernel: each 512-word tile coded by its own wave from the run
//           carries it reads back from the input, sizes then writes); units the tile
//           table cannot hold go to encode_tiled_kernel (tile by tile, one wave).
//   decode  the record chain (tag -> record length -> next tag) is serial. Small:
//           decode_small_kernel, lane per unit. Mid, in large batches: the words decoder
//           (decode_words_kernel): lane per unit, quad-coalesced loads into an
//           LDS ring, one output word per step, staged in 128-B LDS lines and stored by
//           eight lanes per line. Otherwise two passes: pass 1 (decode_index_kernel) walks
//           every unit's chain once, lane per unit, with the same ring loads, and leaves
//           one u16 record per 16-B piece; pass 2 (decode_fill_kernel, wave per unit)
//           starts every lane at its own pieces' first tag, lists the source of each
//           output word (runs' later words filled by a wave scan) and expands with
//           coalesced stores. Long: window-parallel
//           (long_windows / window_spec / window_resolve / window_fill: 4608-B windows
//           speculated from every entry state, resolved in order per unit, expanded in
//           parallel); units the window table cannot hold go to decode_wave_kernel
//           (wave per unit, window by window). The size pass (estimateUnpackedSize) is
//           the index walk without records for mid units and window_spec / window_resolve
//           for long ones.
//   also    Reader.readPackedMessage batched (read_header_kernel + gated index / fill
//           passes), framing fused with encode (encode_message_kernel), Message.init
//           (message_init_kernel), Message.validate (validate_kernel), synthetic data
//           (generate_kernel) and the offsets scan.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "capnp_packed.h"
#include "kernels.h"

namespace cpk {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// ---- encode fast path ------------------------------------------------------
constexpr uint32_t kEncMaxWords = 512;                 // 4 KiB unpacked unit
constexpr uint32_t kEncRow = 80;                       // 64 B words + 16 B pad per lane row
constexpr uint32_t kEncLds = 64 * kEncRow;             // 5120 B; reused for the packed output
// max packed size of 512 words is 9*512+1 = 4609 B; + 16 B align slack + 16 B round-up <= 5120

enum : int32_t {
    ST_OK = CAPNP_PACKED_OK,
    ST_SIZE = CAPNP_PACKED_INVALID_MESSAGE_SIZE,
    ST_EOF = CAPNP_PACKED_UNEXPECTED_EOF,
    ST_SPACE = CAPNP_PACKED_OUT_OF_SPACE,
    ST_ARG = CAPNP_PACKED_INVALID_ARGUMENT,
    ST_DEVERR = CAPNP_PACKED_DEVICE_ERROR,  // a kernel's own loop guard tripped (never expected)
    // Reader.readPackedMessage (reader.zig:84-156)
    ST_EOS = CAPNP_PACKED_END_OF_STREAM,
    ST_SEGCOUNT = CAPNP_PACKED_INVALID_SEGMENT_COUNT,
    ST_SEGLIMIT = CAPNP_PACKED_SEGMENT_COUNT_LIMIT_EXCEEDED,
    ST_TOOLARGE = CAPNP_PACKED_MESSAGE_TOO_LARGE,
    ST_OVERSHOOT = CAPNP_PACKED_INVALID_PACKED_MESSAGE,
    ST_TRUNC = CAPNP_PACKED_TRUNCATED_MESSAGE,  // Message.init (message.zig:353/380)
    // Message.validate (message.zig:699-969)
    ST_EMPTY = CAPNP_PACKED_EMPTY_MESSAGE,
    ST_NEST = CAPNP_PACKED_NESTING_LIMIT_EXCEEDED,
    ST_SEGID = CAPNP_PACKED_INVALID_SEGMENT_ID,
    ST_PTR = CAPNP_PACKED_INVALID_POINTER,
    ST_OOB = CAPNP_PACKED_OUT_OF_BOUNDS,
    ST_TRAV = CAPNP_PACKED_TRAVERSAL_LIMIT_EXCEEDED,
    ST_FAR = CAPNP_PACKED_INVALID_FAR_POINTER,
    ST_ICP = CAPNP_PACKED_INVALID_INLINE_COMPOSITE_POINTER,
    ST_LIST = CAPNP_PACKED_LIST_TOO_LARGE,
};
// internal status between decode passes: the unit goes to a full (fallback) decoder
constexpr int32_t kStNeedFull = 0x7FFF0001;
constexpr int32_t kStNeedWalk = 0x7FFF0002;  // read-message: the one-pass walk could not take the unit
constexpr int32_t kStNeedGate = 0x7FFF0003;  // read-message: walked (consumed known), records next
constexpr int32_t kStWords = 0x7FFF0005;     // read-message: the words decoder's (read_header_kernel)
constexpr uint64_t kRdWordsMax = 1024;       // read-message: framed words the words decoder takes
// status of a long unit between its listing and its worker's result
constexpr int32_t kStPending = CAPNP_PACKED_DEVICE_ERROR;

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16 readable bytes for load lanes that have nothing to stage, and 16 writable
// bytes for the piece-record stores of lanes without a unit.
__device__ __attribute__((aligned(16))) uint8_t cpk_dummy16[16];
__device__ __attribute__((aligned(16))) uint8_t cpk_sink16[16];
__device__ __attribute__((aligned(64))) uint8_t cpk_sink64[64];

// 16-B load of data read for the last time (non-temporal). The fill pass's piece loads
// use it (decode 2.42 -> 2.40 ms); encode's staging loads were slower with it.
__device__ __forceinline__ uint4 load_nt(const void* p) {
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
}

// Ring loads of the lane-per-unit
// decoders in inline asm, so hipcc neither turns them into FLAT instructions
// (pointers that went through __shfl / LDS lose their address space, and FLAT counts on
// lgkmcnt too: every LDS wait of the walk would wait for the prefetch) nor waits for them
// itself (its own vmcnt(0) before the ring writes would also wait for the previous round's
// stores). The kernels count them (s_waitcnt vmcnt(N)) and pin the loaded registers after
// the wait (cdna_hip_programming.md §5.7 item 1, form ii).
__device__ __forceinline__ void ds_gload16(u32x4& d, const void* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}

// LDS-DMA: each lane's 16 B at gsrc straight into LDS at lds_base + 16 * lane (no VGPR
// destination; count it with vmcnt, then a barrier before other waves read it). M0 is written
// and restored in the same statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
}
// the LDS byte address of a __shared__ object
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t*)p);
}

// Order LDS traffic between lanes of ONE wave (the wave owns its LDS slice).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// a 64-bit value from lane `src` (two 32-bit shuffles, zero-extended halves: an int | u64 would
// sign-extend the low half)
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, uint32_t src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}


// Wave scans on DPP: row_shr:1/2/4/8 inside each 16-lane row, then row_bcast:15 and
// row_bcast:31 across rows (gfx9). A lane a step does not reach keeps `ident`. No LDS
// round trips (the ds_bpermute scans they replace cost ~6 LDS latencies in a row).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v, uint32_t ident) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, CTRL, ROWS, 0xF, false);
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, uint32_t /*lane*/) {
    v += dpp_mov<0x111, 0xF>(v, 0u);
    v += dpp_mov<0x112, 0xF>(v, 0u);
    v += dpp_mov<0x114, 0xF>(v, 0u);
    v += dpp_mov<0x118, 0xF>(v, 0u);
    v += dpp_mov<0x142, 0xA>(v, 0u);
    v += dpp_mov<0x143, 0xC>(v, 0u);
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v, uint32_t /*lane*/) {
    v = max(v, dpp_mov<0x111, 0xF>(v, 0u));
    v = max(v, dpp_mov<0x112, 0xF>(v, 0u));
    v = max(v, dpp_mov<0x114, 0xF>(v, 0u));
    v = max(v, dpp_mov<0x118, 0xF>(v, 0u));
    v = max(v, dpp_mov<0x142, 0xA>(v, 0u));
    v = max(v, dpp_mov<0x143, 0xC>(v, 0u));
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_min(uint32_t v) {
    v = min(v, dpp_mov<0x111, 0xF>(v, ~0u));
    v = min(v, dpp_mov<0x112, 0xF>(v, ~0u));
    v = min(v, dpp_mov<0x114, 0xF>(v, ~0u));
    v = min(v, dpp_mov<0x118, 0xF>(v, ~0u));
    v = min(v, dpp_mov<0x142, 0xA>(v, ~0u));
    v = min(v, dpp_mov<0x143, 0xC>(v, ~0u));
    return v;
}

// sum of a u64 over the wave (DPP steps on both halves, 64-bit adds)
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#define CPK_SUM64_STEP(CTRL, ROWS)                                                              \
    v += (uint64_t)dpp_mov<CTRL, ROWS>((uint32_t)v, 0u) | ((uint64_t)dpp_mov<CTRL, ROWS>((uint32_t)(v >> 32), 0u) << 32)
    CPK_SUM64_STEP(0x111, 0xF);
    CPK_SUM64_STEP(0x112, 0xF);
    CPK_SUM64_STEP(0x114, 0xF);
    CPK_SUM64_STEP(0x118, 0xF);
    CPK_SUM64_STEP(0x142, 0xA);
    CPK_SUM64_STEP(0x143, 0xC);
#undef CPK_SUM64_STEP
    return (uint64_t)__builtin_amdgcn_readlane((uint32_t)v, kWave - 1) |
           ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), kWave - 1) << 32);
}

// the previous lane's v (wave_shr:1); lane 0 gets ident
__device__ __forceinline__ uint32_t wave_prev_lane(uint32_t v, uint32_t ident) { return dpp_mov<0x138, 0xF>(v, ident); }

// Lane l - 1's v (lane 0: 0), read with every lane active: the asm pins the DPP move (and
// the computation of v) in front of any branch on the lane, since a DPP read of a lane the
// EXEC mask excludes returns that lane's stale register.
__device__ __forceinline__ uint32_t fu_prev_lane(uint32_t v) {
    uint32_t r = dpp_mov<0x138, 0xF>(v, 0u);
    asm volatile("" : "+v"(r));
    return r;
}

// v of the first lane above this one with `has` set, or `none` (encode_tile's run ends)
__device__ __forceinline__ uint32_t next_break(bool has, uint32_t v, uint32_t lane, uint32_t none) {
    const uint64_t above = (__builtin_amdgcn_ballot_w64(has) >> lane) >> 1;  // lanes > this one
    const uint32_t src = above ? lane + 1u + (uint32_t)__builtin_ctzll(above) : lane;
    const uint32_t r = (uint32_t)__shfl((int)v, (int)src, kWave);
    return above ? r : none;
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return __builtin_amdgcn_readlane(v, l);
}

// Zero-byte tag of a little-endian word: bit k set <=> byte k != 0
// (message.zig:257-262 builds the same tag byte-by-byte).
__device__ __forceinline__ uint32_t nonzero_tag32(uint32_t x) {
    uint32_t y = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;   // byte high bit <=> byte != 0
    return ((y & 0x80808080u) * 0x00204081u) >> 28;        // gather the 4 high bits
}
__device__ __forceinline__ uint32_t nonzero_tag(uint64_t w) {
    // byte k of c: bit 0 = byte k nonzero, bit 4 = byte k + 4 nonzero; the dot product with
    // 2^k gathers them (one full-rate v_dot4 instead of two quarter-rate multiplies)
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t yl = ((lo & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | lo, yh = ((hi & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | hi;
    const uint32_t c = ((yl >> 7) & 0x01010101u) | ((yh >> 3) & 0x10101010u);
    return __builtin_amdgcn_udot4(c, 0x08040201u, 0u, false);
}

// v_perm_b32 over the 8 bytes of d: selector byte r in 0..7 picks byte r, 0x0C gives 0.
__device__ __forceinline__ uint64_t perm64(uint64_t d, uint64_t sel) {
    uint32_t lo = (uint32_t)d, hi = (uint32_t)(d >> 32);
    uint32_t a = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
    uint32_t b = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
    return (uint64_t)a | ((uint64_t)b << 32);
}

// v_perm_b32 selector tables, built at compile time (a block copies one into LDS):
//   compact: gathers the nonzero bytes of a word with tag t into bytes 0..popc-1
//            (0x0C = zero above them);
//   expand:  scatters popc(t) packed bytes back to the set-bit positions of t.
struct alignas(16) SelLut {
    uint64_t v[256];
};
constexpr SelLut make_sel_lut(bool expand) {
    SelLut lut{};
    for (uint32_t t = 0; t < 256; ++t) {
        uint64_t sel = expand ? 0ull : 0x0C0C0C0C0C0C0C0CULL;
        uint32_t r = 0;
        for (uint32_t k = 0; k < 8; ++k) {
            const bool set = (t >> k) & 1u;
            if (expand) {
                sel |= (set ? (uint64_t)(r++) : 0x0Cull) << (8 * k);
            } else if (set) {
                sel = (sel & ~(0xFFULL << (8 * r))) | ((uint64_t)k << (8 * r));
                ++r;
            }
        }
        lut.v[t] = sel;
    }
    return lut;
}
__device__ constexpr SelLut kCompactLut = make_sel_lut(false);
__device__ constexpr SelLut kExpandLut = make_sel_lut(true);
// The compact selector moved up one byte (byte 0 selects a zero byte): perm64(w, it) is the
// tag's record payload at bytes 1..popc, ready to OR with the tag (encode_tile).
__device__ __forceinline__ uint64_t compact_selector(uint32_t t) { return (kCompactLut.v[t] << 8) | 0x0Cull; }
// the same as a table, for a copy into LDS by LDS-DMA (encode_kernel)
constexpr SelLut make_compact_sel() {
    SelLut l = make_sel_lut(false);
    for (uint32_t t = 0; t < 256; ++t) l.v[t] = (l.v[t] << 8) | 0x0Cull;
    return l;
}
__device__ constexpr SelLut kCompactSel = make_compact_sel();
__device__ __forceinline__ uint64_t expand_selector(uint32_t t) { return kExpandLut.v[t]; }

// Unaligned 8-byte read from an LDS byte array (two aligned ds_read_b64 + funnel).
__device__ __forceinline__ uint64_t lds_read_u64_unaligned(const uint8_t* base, uint32_t p) {
    uint32_t a = p & ~7u;
    uint64_t lo = *reinterpret_cast<const uint64_t*>(base + a);
    uint64_t hi = *reinterpret_cast<const uint64_t*>(base + a + 8);
    uint32_t sh = (p & 7u) * 8u;
    return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
}

// Stage nch 16-B chunks from global g[0 .. 16*nch) into lds[0 .. 16*nch):
// lane l moves chunks l, l+64, ... Loads AND stores are unconditional, with the
// chunk index clamped to nch-1 (a clamped lane re-writes the last chunk with the
// same bytes), so the compiler cannot sink the loads into guarded blocks: all K
// loads are in flight together and one vmcnt wait lands them.
template <int K>
__device__ __forceinline__ void stage_linear(uint8_t* lds, const uint8_t* g, uint32_t nch, uint32_t lane) {
    if (nch == 0) return;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = min(lane + 64u * k, nch - 1);
        v[k] = *reinterpret_cast<const uint4*>(g + 16 * (uint64_t)c);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t c = min(lane + 64u * k, nch - 1);
        *reinterpret_cast<uint4*>(lds + 16 * c) = v[k];
    }
}

// expand: packed bytes d (byte r = r-th nonzero byte) -> word with zeros where tag bit is clear
__device__ __forceinline__ uint64_t expand_word(uint64_t d, uint32_t t) {
    const uint32_t s_lo = ((t & 0xFu) * 0x00204081u) & 0x01010101u;        // byte k = bit k
    const uint32_t s_hi = (((t >> 4) & 0xFu) * 0x00204081u) & 0x01010101u;
    const uint32_t inc_lo = s_lo * 0x01010101u;                             // inclusive byte prefix sums
    const uint32_t inc_hi = s_hi * 0x01010101u + (inc_lo >> 24) * 0x01010101u;
    const uint32_t m_lo = s_lo * 0xFFu, m_hi = s_hi * 0xFFu;
    const uint32_t sel_lo = ((inc_lo - s_lo) & m_lo) | (0x0C0C0C0Cu & ~m_lo);
    const uint32_t sel_hi = ((inc_hi - s_hi) & m_hi) | (0x0C0C0C0Cu & ~m_hi);
    return perm64(d, (uint64_t)sel_lo | ((uint64_t)sel_hi << 32));
}

// ---------------------------------------------------------------------------
// Serial per-wave fallback (lane 0), any unit size. Restates message.zig
// directly over global memory. Used for units beyond the fast-path limits.
// ---------------------------------------------------------------------------

// Bytes [lo, hi) (0 <= lo < hi <= 16) of a 16-B chunk (x0 = bytes 0-7, x1 = bytes 8-15)
// whose 16-B aligned home is c16: naturally aligned 1/2/4/8-B stores, up to 8-B alignment
// and then down from it (at most 8 predicated stores). A byte loop runs to the wave's
// longest partial chunk (C5 small encode: ~100 us of 400).
__device__ __forceinline__ void store_partial16(uint8_t* c16, uint32_t lo, uint32_t hi, uint64_t x0, uint64_t x1) {
    auto put = [&](uint32_t sz) {  // bytes [lo, lo + sz), lo aligned to sz
        const uint64_t v = lo < 8 ? x0 >> (8 * lo) : x1 >> (8 * (lo - 8));
        uint8_t* const p = c16 + lo;
        if (sz == 8) *reinterpret_cast<uint64_t*>(p) = v;
        else if (sz == 4) *reinterpret_cast<uint32_t*>(p) = (uint32_t)v;
        else if (sz == 2) *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;
        else *p = (uint8_t)v;
        lo += sz;
    };
    if ((lo & 1) && lo + 1 <= hi) put(1);
    if ((lo & 2) && lo + 2 <= hi) put(2);
    if ((lo & 4) && lo + 4 <= hi) put(4);
    if (lo + 8 <= hi) put(8);
    if (lo + 4 <= hi) put(4);
    if (lo + 2 <= hi) put(2);
    if (lo + 1 <= hi) put(1);
}

__device__ __forceinline__ uint64_t gload64(const uint8_t* p) {  // 8-aligned
    return *reinterpret_cast<const uint64_t*>(p);
}
__device__ __forceinline__ int word_has_zero_byte(uint64_t v) {  // message.zig:196-198
    return ((v - 0x0101010101010101ULL) & ~v & 0x8080808080808080ULL) != 0;
}

// message.zig:200-271; when out == nullptr only the size is computed.
__device__ uint64_t serial_pack(const uint8_t* in, uint64_t words, uint8_t* out) {
    uint64_t o = 0, i = 0;
    while (i < words) {
        uint64_t w = gload64(in + 8 * i);
        if (w == 0) {
            uint64_t run = 1;
            while (run < 256 && i + run < words && gload64(in + 8 * (i + run)) == 0) ++run;
            if (out) { out[o] = 0; out[o + 1] = (uint8_t)(run - 1); }
            o += 2;
            i += run;
            continue;
        }
        if (!word_has_zero_byte(w)) {
            uint64_t run = 1;
            while (run < 256 && i + run < words && !word_has_zero_byte(gload64(in + 8 * (i + run)))) ++run;
            if (out) {
                out[o] = 0xFF;
                for (int k = 0; k < 8; ++k) out[o + 1 + k] = (uint8_t)(w >> (8 * k));
                out[o + 9] = (uint8_t)(run - 1);
                for (uint64_t b = 0; b < 8 * (run - 1); ++b) out[o + 10 + b] = in[8 * (i + 1) + b];
            }
            o += 10 + 8 * (run - 1);
            i += run;
            continue;
        }
        uint32_t tag = 0, nz = 0;
        for (int k = 0; k < 8; ++k) {
            uint8_t b = (uint8_t)(w >> (8 * k));
            if (b) {
                tag |= 1u << k;
                if (out) out[o + 1 + nz] = b;
                ++nz;
            }
        }
        if (out) out[o] = (uint8_t)tag;
        o += 1 + nz;
        i += 1;
    }
    return o;
}

// message.zig:152-191; returns ST_OK / ST_EOF and the decoded size.
__device__ int32_t serial_decoded_size(const uint8_t* p, uint64_t n, uint64_t* size) {
    uint64_t i = 0, total = 0;
    while (i < n) {
        uint32_t t = p[i++];
        if (t == 0x00) {
            if (i >= n) return ST_EOF;
            total += 8 * (1 + (uint64_t)p[i++]);
        } else if (t == 0xFF) {
            if (i + 8 > n) return ST_EOF;
            i += 8;
            if (i >= n) return ST_EOF;
            uint64_t c = p[i++];
            if (i + 8 * c > n) return ST_EOF;
            total += 8 * (1 + c);
            i += 8 * c;
        } else {
            uint32_t k = __popc(t);
            if (i + k > n) return ST_EOF;
            total += 8;
            i += k;
        }
    }
    *size = total;
    return ST_OK;
}

// message.zig:97-142 (input already validated by serial_decoded_size).
__device__ void serial_unpack(const uint8_t* p, uint64_t n, uint8_t* out) {
    uint64_t i = 0, o = 0;
    while (i < n) {
        uint32_t t = p[i++];
        if (t == 0x00) {
            uint64_t z = 8 * (1 + (uint64_t)p[i++]);
            for (uint64_t b = 0; b < z; ++b) out[o + b] = 0;
            o += z;
        } else if (t == 0xFF) {
            for (int b = 0; b < 8; ++b) out[o + b] = p[i + b];
            o += 8;
            i += 8;
            uint64_t c = p[i++];
            for (uint64_t b = 0; b < 8 * c; ++b) out[o + b] = p[i + b];
            o += 8 * c;
            i += 8 * c;
        } else {
            for (int k = 0; k < 8; ++k) out[o + k] = ((t >> k) & 1u) ? p[i++] : 0;
            o += 8;
        }
    }
}

// ---------------------------------------------------------------------------
// ENCODE
// ---------------------------------------------------------------------------
// One wave encodes one 512-word (4 KiB) tile of a unit: encode_tile. A unit of at
// most 512 words is a single tile (the headline path). Longer units are walked by
// the same wave tile after tile (encode_kernel's tiled loop), with two carries:
//   run starts (cz, cf): the start of the zero-class / literal-class run that is
//     still open at the tile start, so a run continuing from earlier tiles keeps
//     its 256-word head positions (message.zig:211-225 / 231-251);
//   lookahead (nbz, nbf): the first Z / F break at or after the tile end (first
//     non-zero word / first word with a zero byte), read from the next tile, so a
//     head near the tile end gets its count min(256, run end - i) - 1; a break
//     more than 256 words ahead cannot change a count, so 256 words suffice.

// Stage words [0, words) of src (8-aligned) into the row layout: word w at
// lds[(w >> 3) * kEncRow + (w & 7) * 8]. Split in two so a persistent wave can have the
// next unit's loads in flight while it codes the current one (encode_kernel).
__device__ __forceinline__ void encode_load(uint4 (&v)[5], const uint8_t* src, uint32_t words, uint32_t lane) {
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);  // 0 or 8
    const uint8_t* g = src - s;
    const uint32_t nch = (s + 8 * words + 15) >> 4;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if ((uint32_t)(64 * k) < nch) {
            uint32_t c = min(lane + 64u * k, nch - 1);
            v[k] = *reinterpret_cast<const uint4*>(g + 16 * (uint64_t)c);  // (non-temporal: slower, 1.52 -> 1.72 ms)
        }
    }
}
__device__ __forceinline__ void encode_put(uint8_t* lds, const uint4 (&v)[5], uint32_t s, uint32_t words,
                                           uint32_t lane) {
    const uint32_t nch = (s + 8 * words + 15) >> 4;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        uint32_t c = lane + 64 * k;
        if ((uint32_t)(64 * k) < nch && c < nch) {
            if (s == 0) {
                uint32_t w = 2 * c;
                *reinterpret_cast<uint4*>(lds + (w >> 3) * kEncRow + (w & 7) * 8) = v[k];
            } else {
                uint64_t lo = (uint64_t)v[k].x | ((uint64_t)v[k].y << 32);
                uint64_t hi = (uint64_t)v[k].z | ((uint64_t)v[k].w << 32);
                if (c > 0) {
                    uint32_t w = 2 * c - 1;
                    *reinterpret_cast<uint64_t*>(lds + (w >> 3) * kEncRow + (w & 7) * 8) = lo;
                }
                uint32_t w = 2 * c;
                if (w < words) *reinterpret_cast<uint64_t*>(lds + (w >> 3) * kEncRow + (w & 7) * 8) = hi;
            }
        }
    }
}
// encode_put for a payload that starts at framed word w0 (after a message's segment table): the
// 16-B chunks land as two 8-B words each (w0 + word may be odd)
__device__ __forceinline__ void encode_put_at(uint8_t* lds, const uint4 (&v)[5], uint32_t s, uint32_t words,
                                              uint32_t lane, uint32_t w0) {
    const uint32_t nch = (s + 8 * words + 15) >> 4;
    auto put8 = [&](uint32_t w, uint64_t x) {
        const uint32_t f = w0 + w;
        *reinterpret_cast<uint64_t*>(lds + (f >> 3) * kEncRow + (f & 7) * 8) = x;
    };
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t c = lane + 64 * k;
        if ((uint32_t)(64 * k) < nch && c < nch) {
            const uint64_t lo = (uint64_t)v[k].x | ((uint64_t)v[k].y << 32);
            const uint64_t hi = (uint64_t)v[k].z | ((uint64_t)v[k].w << 32);
            if (s == 0) {
                put8(2 * c, lo);
                if (2 * c + 1 < words) put8(2 * c + 1, hi);
            } else {
                if (c > 0) put8(2 * c - 1, lo);
                if (2 * c < words) put8(2 * c, hi);
            }
        }
    }
}
__device__ __forceinline__ void encode_stage(uint8_t* lds, const uint8_t* src, uint32_t words, uint32_t lane) {
    uint4 v[5];
    encode_load(v, src, words, lane);
    encode_put(lds, v, (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15), words, lane);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_incl_min(v), kWave - 1);
}

// First Z break and first F break among words [0, nw) of src, nw <= 256, as
// offsets (nw when there is none); wave-uniform results.
__device__ __forceinline__ void encode_lookahead(const uint8_t* src, uint32_t nw, uint32_t lane, uint32_t& bz,
                                                 uint32_t& bf) {
    uint32_t fz = nw, ff = nw;
#pragma unroll
    for (int t = 3; t >= 0; --t) {
        const uint32_t i = 4 * lane + t;
        if (i < nw) {
            const uint32_t tg = nonzero_tag(*reinterpret_cast<const uint64_t*>(src + 8 * i));
            if (tg != 0) fz = i;
            if (tg != 0xFF) ff = i;
        }
    }
    bz = wave_min(fz);
    bf = wave_min(ff);
}

// Encode one staged tile: words [tb, tb + words) of the unit (absolute word
// indices; tb = 0 for a single tile). SINGLE: the whole unit (no carries; run
// crossings are tested per lane boundary). Returns the tile's packed size; writes
// the packed bytes to dst when WRITE and they fit in `room`.
template <bool WRITE, bool SINGLE, bool FULL = false>
__device__ __forceinline__ uint32_t encode_tile(uint8_t* lds, const uint64_t* lut, uint32_t lane, uint32_t words,
                                                uint32_t tb, uint32_t& cz_c, uint32_t& cf_c, uint32_t nbz,
                                                uint32_t nbf, uint8_t* dst, uint64_t room,
                                                const uint8_t* direct = nullptr, const uint4* pre = nullptr) {
    const uint32_t wend = tb + words;  // absolute end of the tile
    // ---- lane j owns words [tb + 8j, tb + 8j + 8) --------------------------------
    const uint32_t base = tb + lane * 8;
    // FULL: a 512-word tile, every lane owns 8 words (the per-word range tests fold away)
    const uint32_t nw = FULL ? 8u : (lane * 8 < words ? min(8u, words - lane * 8) : 0u);
    uint64_t w[8];
    if (FULL && pre) {  // the lane's 64 B, loaded by the caller before the block's barrier
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[2 * q] = (uint64_t)pre[q].x | ((uint64_t)pre[q].y << 32);
            w[2 * q + 1] = (uint64_t)pre[q].z | ((uint64_t)pre[q].w << 32);
        }
    } else if (FULL && direct) {  // a 16-B aligned full tile: the lane's 64 B straight from memory
        const uint4* row = reinterpret_cast<const uint4*>(direct + 64 * lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 r = row[q];
            w[2 * q] = (uint64_t)r.x | ((uint64_t)r.y << 32);
            w[2 * q + 1] = (uint64_t)r.z | ((uint64_t)r.w << 32);
        }
    } else if (FULL || nw) {
        const uint4* row = reinterpret_cast<const uint4*>(lds + lane * kEncRow);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint4 r = row[q];
            w[2 * q] = (uint64_t)r.x | ((uint64_t)r.y << 32);
            w[2 * q + 1] = (uint64_t)r.z | ((uint64_t)r.w << 32);
        }
    } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) w[t] = 0;
    }

    uint32_t tag[8];
    uint32_t zmask = 0, fmask = 0;  // bit t: word t is all-zero / has no zero byte
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        tag[t] = nonzero_tag(w[t]);
        const bool in = FULL || (uint32_t)t < nw;  // selects, not branches: the per-word
        zmask |= (in && tag[t] == 0) ? 1u << t : 0u;     // logic stays off the exec mask
        fmask |= (in && tag[t] == 0xFF) ? 1u << t : 0u;
    }
    // break positions for the zero-run (Z) and literal-run (F) classes: last break + 1
    // (seeded with the carried run start) and first break (seeded with the lookahead)
    uint32_t lbz = cz_c, lbf = cf_c, fbz = nbz, fbf = nbf;
#pragma unroll
    for (int t = 7; t >= 0; --t) {
        const uint32_t i = base + t;
        const bool in = FULL || (uint32_t)t < nw;
        const bool bz = in && !((zmask >> t) & 1u), bf = in && !((fmask >> t) & 1u);
        lbz = bz ? max(lbz, i + 1) : lbz;
        fbz = bz ? i : fbz;
        lbf = bf ? max(lbf, i + 1) : lbf;
        fbf = bf ? i : fbf;
    }
    // run start carried into this lane = last break before it (+1); run end = first break after it.
    // In a single tile where no zero run and no literal run crosses a lane boundary (the
    // common case away from very sparse or very dense data) the carries are the lane's
    // own bounds and the four wave scans are skipped.
    uint32_t cz = base, cf = base, ez = min(base + 8, wend), ef = ez;
    bool scan = true;
    if (SINGLE) {
        const uint64_t bz0 = __ballot(zmask & 1u), bz7 = __ballot((zmask >> 7) & 1u);
        const uint64_t bf0 = __ballot(fmask & 1u), bf7 = __ballot((fmask >> 7) & 1u);
        scan = ((bz0 & (bz7 << 1)) | (bf0 & (bf7 << 1))) != 0;
    }
    if (scan) {
        cz = wave_prev_lane(wave_incl_max(lbz, lane), 0u);
        cf = wave_prev_lane(wave_incl_max(lbf, lane), 0u);
        // run end: the first break of the next lane that holds one (a lane's fb is its first
        // break, or the lookahead, which lies past every break of the tile): a ballot and one
        // shuffle instead of a six-step suffix-min scan
        ez = next_break(fbz != nbz, fbz, lane, nbz);
        ef = next_break(fbf != nbf, fbf, lane, nbf);
        if (lane == 0) { cz = cz_c; cf = cf_c; }
    }
    // carries for the next tile: the run starts open at the tile end
    uint32_t lz_all = 0, lf_all = 0;
    if (!SINGLE) {
        lz_all = readlane(wave_incl_max(lbz, lane), 63);
        lf_all = readlane(wave_incl_max(lbf, lane), 63);
    }

    uint32_t rs[8];  // run start of word t's class run (Z or F)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        uint32_t i = base + t;
        rs[t] = ((zmask >> t) & 1u) ? cz : cf;
        if (!((zmask >> t) & 1u)) cz = i + 1;
        if (!((fmask >> t) & 1u)) cf = i + 1;
    }
    uint32_t re[8];  // run end (first break after word t) of its class
#pragma unroll
    for (int t = 7; t >= 0; --t) {
        uint32_t i = base + t;
        re[t] = ((zmask >> t) & 1u) ? ez : ef;
        const bool in = FULL || (uint32_t)t < nw;
        ez = (in && !((zmask >> t) & 1u)) ? i : ez;
        ef = (in && !((fmask >> t) & 1u)) ? i : ef;
    }
    uint32_t sz[8], cnt[8];
    uint32_t total = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        uint32_t i = base + t;
        uint32_t head = ((i - rs[t]) & 255u) == 0;
        cnt[t] = min(256u, re[t] - i) - 1;  // message.zig:214-223 / 236-245
        // 00: 2 bytes at a head, else 0; FF: 10 / 8; other tags: 1 + popc (zero / FF words
        // are exclusive, popc 0 / 8)
        uint32_t s = __popc(tag[t]) + (((zmask | fmask) >> t) & 1u ? (head ? 2u : 0u) : 1u);
        if (!FULL) s = (uint32_t)t < nw ? s : 0u;
        sz[t] = s;
        total += s;
    }
    const uint32_t incl = wave_incl_sum(total, lane);
    const uint32_t P = readlane(incl, 63);
    const uint32_t o = incl - total;
    cz_c = lz_all;
    cf_c = lf_all;
    if (!WRITE || (uint64_t)P > room) return P;

    // ---- assemble the packed bytes in LDS (reusing the staging slice) -------------
    const uint32_t so = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15);
    const uint32_t nch_out = (so + P + 15) >> 4;
    wave_lds_sync();  // every lane has its words in registers
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        uint32_t c = lane + 64 * k;
        if (c < nch_out) *reinterpret_cast<uint4*>(lds + 16 * c) = make_uint4(0, 0, 0, 0);
    }
    wave_lds_sync();
    {
        // Each record (<= 10 bytes) is OR-ed into the zeroed buffer as two (FF heads:
        // three) aligned u64 pieces: no per-byte shifting state, no branches. A word with
        // no bytes (a zero run's body, a word past the tile) ORs zeros; every address stays
        // inside the slice (P <= 9 bytes per word: at most ~4.6 KB of the 5 KB).
        const uint32_t x0 = so + o;
        uint32_t x = x0, ex = 0;  // ex bit t: an FF head whose count byte opens a third u64
        // lanes past a short unit's words skip the ORs (one branch per lane, not per word:
        // C5's mid units leave most lanes of a wave without words)
        if (FULL || nw != 0)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            // tag + nonzero bytes (00: just the tag; FF: the tag and bytes 0..6 of an FF head)
            uint64_t sel = lut[tag[t]];
            asm volatile("" : "+v"(sel));  // read for every word: the selects below stay branch-free
            const uint64_t rec = (uint64_t)tag[t] | perm64(w[t], sel);
            const bool zt = (zmask >> t) & 1u, head = sz[t] == 10u;  // head: FF w0..w7 <count>
            const bool body = ((fmask >> t) & 1u) && !head;          // a literal run's body word
            uint64_t lo = rec | ((uint64_t)(zt ? cnt[t] : 0u) << 8);    // 00 <count>
            lo = body ? w[t] : lo;
            lo = sz[t] ? lo : 0ull;
            const uint64_t hi = head ? ((w[t] >> 56) | ((uint64_t)cnt[t] << 8)) : 0ull;
            const uint32_t a = x & ~7u, sh = (x & 7u) * 8u;
            atomicOr(reinterpret_cast<unsigned long long*>(lds + a), (unsigned long long)(lo << sh));
            atomicOr(reinterpret_cast<unsigned long long*>(lds + a + 8),
                     (unsigned long long)(((lo >> 1) >> (63u - sh)) | (hi << sh)));
            ex |= (sh == 56 && (hi >> 8)) ? 1u << t : 0u;
            x += sz[t];
        }
        if (__builtin_amdgcn_ballot_w64(ex != 0) != 0) {  // rare (FF heads at byte 7 of a u64)
            x = x0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if ((ex >> t) & 1u)
                    atomicOr(reinterpret_cast<unsigned long long*>(lds + (x & ~7u) + 16),
                             (unsigned long long)(((w[t] >> 56) | ((uint64_t)cnt[t] << 8)) >> 8));
                x += sz[t];
            }
        }
    }
    wave_lds_sync();

    // ---- coalesced write-back ------------------------------------------------------
    {
        uint8_t* gdst = dst - so;  // 16-B aligned
        const uint32_t lo = so, hi = so + P;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint32_t c = lane + 64 * k;
            if (c < nch_out) {
                uint32_t cb = 16 * c, ce = cb + 16;
                if (cb >= lo && ce <= hi) {
                    // streaming output: non-temporal (nothing re-reads it from L2 in this pass)
                    __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(lds + cb),
                                                reinterpret_cast<u32x4*>(gdst + cb));
                } else {
                    const uint32_t a = max(cb, lo), e = min(ce, hi);  // the unit's first / last chunk
                    store_partial16(gdst + cb, a - cb, e - cb, *reinterpret_cast<const uint64_t*>(lds + cb),
                                    *reinterpret_cast<const uint64_t*>(lds + cb + 8));
                }
            }
        }
    }
    return P;
}

// A unit's input offset and length, and, for an aligned 512-word unit (every unit of the
// headline: DIRECT), the lane's 64 B, loaded by encode_kernel before its selector-table barrier.
struct EncPre {
    uint64_t b0, nbytes;
    uint4 r[4];
};

// One unit of encode_kernel (wave-uniform `unit`), from its prefetched metadata.
template <bool WRITE, bool DIRECT>
__device__ __forceinline__ void encode_unit(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                      const uint64_t* __restrict__ out_off,
                                                      const uint64_t* __restrict__ out_cap,
                                                      uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                      uint32_t unit, uint8_t* lds, const uint64_t* lut,
                                                      uint32_t lane, const EncPre& pre) {
    const uint64_t b0 = pre.b0;
    const uint64_t nbytes = pre.nbytes;
    uint64_t ob = 0, cap = 0;
    if (WRITE) {
        ob = out_off[unit];
        cap = out_cap[unit];
    }
    int32_t st = ST_OK;
    if (reinterpret_cast<uintptr_t>(in + b0) & 7) st = ST_ARG;
    if (st == ST_OK && (nbytes & 7)) st = ST_SIZE;  // message.zig:201
    if (st != ST_OK) {
        if (lane == 0) { out_len[unit] = 0; status[unit] = st; }
        return;
    }
    const uint8_t* const src = in + b0;
    if (nbytes / 8 > 0xFFFFF000ull) {  // absolute word indices are u32: serial path (> 32 GiB units)
        if (lane == 0) {
            uint64_t P = serial_pack(src, nbytes / 8, nullptr);
            int32_t s2 = ST_OK;
            if (WRITE) {
                if (P > cap) s2 = ST_SPACE;
                else serial_pack(src, nbytes / 8, out + ob);
            }
            out_len[unit] = P;
            status[unit] = s2;
        }
        return;
    }
    const uint32_t words = (uint32_t)(nbytes >> 3);
    if (words <= kEncMaxWords) {  // one tile (the headline 4-KiB units)
        if (!DIRECT) encode_stage(lds, src, words, lane);  // DIRECT: loaded in pre.r
        wave_lds_sync();
        uint32_t cz = 0, cf = 0;
        const uint32_t P = DIRECT ? encode_tile<WRITE, true, true>(lds, lut, lane, words, 0, cz, cf, words, words,
                                                                   out + ob, cap, src, pre.r)
                                  : encode_tile<WRITE, true>(lds, lut, lane, words, 0, cz, cf, words, words, out + ob, cap);
        if (lane == 0) {
            out_len[unit] = P;
            status[unit] = (WRITE && (uint64_t)P > cap) ? ST_SPACE : ST_OK;
        }
    }
    // longer units belong to encode_tiled_kernel, which selects them by the same test
    // (encode_tiled_unit) and may be running beside this kernel on the side stream:
    // nothing of theirs is written here (a separate kernel keeps this one at its
    // register budget)
}

// A wave per unit: the class list's units (launch_encode: the mid units), or the batch.
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void encode_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint64_t* __restrict__ in_len,
                                                        uint32_t n, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint64_t* __restrict__ out_cap,
                                                        uint64_t* __restrict__ out_len,
                                                        int32_t* __restrict__ status,
                                                        const uint32_t* __restrict__ list,
                                                        const uint32_t* __restrict__ list_count) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kEncLds];
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // The selector table goes out first (LDS-DMA by waves 0 and 1, 1 KiB each), then (an aligned
    // 512-word unit, the headline's) the lane's 64 B of the unit; the block barrier waits only for
    // the table, so a block's units are in flight while it lands. The unit's loads are inline asm
    // counted here (a load hipcc knew of would get the barrier's vmcnt(0)); their registers are
    // named in the wait statement itself (cdna_hip_programming.md §5.7 item 1, form ii).
    // a wave per list entry; a list as long as the batch is the identity (class lists keep
    // batch order), so the headline's all-mid batches skip the list read. The grid is sized by
    // the batch, so a short list leaves whole blocks without a unit: they leave at once.
    const uint32_t count = list ? *list_count : n;
    if (blockIdx.x * kWavesPerBlock >= count) return;  // block-uniform
    if (WRITE && wave < 2)
        glds16(reinterpret_cast<const uint8_t*>(&kCompactSel) + 1024u * wave + 16u * lane,
               __builtin_amdgcn_readfirstlane(lds_addr(lut) + 1024u * wave));
    uint8_t* lds = smem + wave * kEncLds;
    const uint32_t slot = blockIdx.x * kWavesPerBlock + wave;
    const bool live = slot < count;  // wave-uniform
    const uint32_t unit = !live ? 0u : (list && count != n) ? __builtin_amdgcn_readfirstlane(list[slot]) : slot;
    EncPre pre;
    pre.b0 = live ? in_off[unit] : 0ull;
    pre.nbytes = live ? in_len[unit] : 0ull;
    const uint8_t* const src = in + pre.b0;
    if (live && pre.nbytes == 8ull * kEncMaxWords && !(reinterpret_cast<uintptr_t>(src) & 15)) {
        const uint4* const row = reinterpret_cast<const uint4*>(src + 64 * lane);
        u32x4 r0, r1, r2, r3;
        ds_gload16(r0, row);
        ds_gload16(r1, row + 1);
        ds_gload16(r2, row + 2);
        ds_gload16(r3, row + 3);
        if (WRITE) {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // the table's DMA, not the unit's loads
            __syncthreads();
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : : "memory");
        pre.r[0] = make_uint4(r0.x, r0.y, r0.z, r0.w);
        pre.r[1] = make_uint4(r1.x, r1.y, r1.z, r1.w);
        pre.r[2] = make_uint4(r2.x, r2.y, r2.z, r2.w);
        pre.r[3] = make_uint4(r3.x, r3.y, r3.z, r3.w);
        encode_unit<WRITE, true>(in, out, out_off, out_cap, out_len, status, unit, lds, lut, lane, pre);
        return;
    }
    if (WRITE) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (!live) return;
    encode_unit<WRITE, false>(in, out, out_off, out_cap, out_len, status, unit, lds, lut, lane, pre);
}

// The units encode_tiled_kernel owns: valid word streams (8-aligned start, whole
// words) of more than one tile, within the u32 word-index range. encode_kernel
// returns early for exactly these, so the two kernels never write the same unit and
// can run concurrently (launch_encode).
__device__ __forceinline__ bool encode_tiled_unit(const uint8_t* in, uint64_t off, uint64_t len) {
    return !(reinterpret_cast<uintptr_t>(in + off) & 7) && !(len & 7) && (len >> 3) > kEncMaxWords &&
           (len >> 3) <= 0xFFFFF000ull;
}

// Long-unit lists (device memory, filled by the class kernels below) for a batch of n
// units: q[0] = long units listed, q[2] = huge units listed (more than kQHuge bytes in);
// the long units at q[kQHead ..] upwards, the huge ones from q[kQHead + n - 1] downwards.
// long_tiles_kernel / long_windows_kernel turn them into the tile / window tables (huge
// units first) and the serial list of units the table could not hold.
constexpr uint64_t kQHuge = 65536;
constexpr uint32_t kQHead = 32;
constexpr uint32_t kClassBlock = 1024;  // units per class-kernel block
constexpr uint32_t kClassK = 12;        // per-block class counters (11 classes used)
__host__ __device__ inline uint64_t class_blocks(uint64_t n) { return (n + kClassBlock - 1) / kClassBlock; }
// u32 index of the serial list (long units no tile / window table could hold)
__host__ __device__ inline uint64_t serial_off(uint64_t n) { return kQHead + 3 * n + kClassK * class_blocks(n); }
__device__ __forceinline__ bool decode_long_unit(const uint8_t* in, uint64_t in_off, uint64_t P, uint8_t* out,
                                                 uint64_t out_off, uint64_t cap);

// Units longer than one tile (encode_tiled_unit) that the tile table could not hold,
// taken from the serial list and encoded one after another, tile by tile.
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void encode_tiled_kernel(const uint8_t* __restrict__ in,
                                                              const uint64_t* __restrict__ in_off,
                                                              const uint64_t* __restrict__ in_len,
                                                              uint32_t n, uint8_t* __restrict__ out,
                                                              const uint64_t* __restrict__ out_off,
                                                              const uint64_t* __restrict__ out_cap,
                                                              uint64_t* __restrict__ out_len,
                                                              int32_t* __restrict__ status, uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kEncLds];
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (q[5] == 0) return;  // no serial units (block-uniform)
    if (WRITE) {
        lut[threadIdx.x] = compact_selector(threadIdx.x);
        __syncthreads();
    }
    uint8_t* lds = smem + wave * kEncLds;
    uint32_t unit = 0;
    // the units long_tiles_kernel could not list (the serial list), one after another
    const uint32_t* const serial = q + serial_off(n);
    for (;;) {  // wave-uniform
    {
        uint32_t i = 0;
        if (lane == 0) i = atomicAdd(q + 10, 1u);
        i = __builtin_amdgcn_readfirstlane(i);
        if (i >= q[5]) break;
        unit = serial[i];
    }
    const uint8_t* const src = in + in_off[unit];
    const uint32_t words = (uint32_t)(in_len[unit] >> 3);
    uint64_t ob = 0, cap = 0;
    if (WRITE) {
        ob = out_off[unit];
        cap = out_cap[unit];
    }
    uint32_t cz = 0, cf = 0;
    uint64_t pos = 0;   // packed bytes so far
    bool fits = true;   // every tile so far was written (WRITE)
    for (uint32_t tb = 0; tb < words; tb += kEncMaxWords) {
        // lane-derived addresses are recomputed per tile, not held across the loops in
        // registers (loop-invariant hoisting had this kernel at 140 VGPRs)
        uint32_t lane_u = lane;
        asm volatile("" : "+v"(lane_u));
        const uint32_t tw = min(kEncMaxWords, words - tb);
        const uint32_t te = tb + tw;
        // the tile's staging loads go out first, so they and the lookahead's loads land
        // together (one memory round trip per tile, not two)
        uint4 v[5];
        encode_load(v, src + 8ull * tb, tw, lane_u);
        uint32_t nbz = words, nbf = words;
        if (te < words) {
            const uint32_t la = min(256u, words - te);
            uint32_t bz, bf;
            encode_lookahead(src + 8ull * te, la, lane_u, bz, bf);
            nbz = bz < la ? te + bz : (la == 256u ? te + 256u : words);
            nbf = bf < la ? te + bf : (la == 256u ? te + 256u : words);
        }
        wave_lds_sync();  // the previous tile's write-back read the slice
        encode_put(lds, v, (uint32_t)(reinterpret_cast<uintptr_t>(src + 8ull * tb) & 15), tw, lane_u);
        wave_lds_sync();
        const uint64_t room = (WRITE && fits && pos <= cap) ? cap - pos : 0;
        const uint32_t Pt = encode_tile<WRITE, false>(lds, lut, lane_u, tw, tb, cz, cf, nbz, nbf, out + ob + pos,
                                                      room);
        if ((uint64_t)Pt > room) fits = false;
        pos += Pt;
    }
    if (lane == 0) {
        out_len[unit] = pos;
        status[unit] = (WRITE && !fits) ? ST_SPACE : ST_OK;
    }
    }  // queued units
}

// ---------------------------------------------------------------------------
// ENCODE straight from segment lists: MessageBuilder.toPackedBytes
// (message.zig:2175-2179 = packPacked(toBytes()), toBytes 2123-2170) without the
// framed copy. One wave per message walks the VIRTUAL framed stream
//   [segment count - 1, size_0 .. size_{c-1}, pad] ++ segment_0 ++ .. ++ segment_{c-1}
// tile by tile through encode_tile (the same carries as encode_tiled_kernel); each
// lane gathers its 8 words of a tile from the header or from the segment that
// holds them (word offsets of the segments in LDS).
// ---------------------------------------------------------------------------
constexpr uint32_t kMsgMaxSegs = 512;  // Message.max_segment_count (message.zig:310)
constexpr uint32_t kMsgOneSegs = 64;   // one-tile pass: a segment per lane (more: the tiled pass)


// PAD (the one-tile pass): the segments' word offsets and addresses live in the 16-B pads of the
// tile's 80-B LDS rows (u32 slot s at row s / 4, bytes 64 + 4 (s % 4); offset s at slot s,
// s <= count, address s at slots 128 + 2s, 129 + 2s), free while the tile is staged: the pass
// needs no LDS beyond encode_kernel's (7 waves per SIMD, not 5), and no global load between the
// segment table and the data.
__device__ __forceinline__ uint8_t* msg_pad(uint8_t* lds, uint32_t slot) {
    return lds + (slot >> 2) * kEncRow + 64 + 4 * (slot & 3);
}
typedef uint64_t u64x2_a8 __attribute__((ext_vector_type(2), aligned(8)));
// Segment data loads through global (AS1) pointers: the addresses come out of LDS, and a
// generic pointer would make FLAT loads, which also count on lgkmcnt (the LDS waits of the
// gather would wait for the data).
__device__ __forceinline__ uint64_t gload8(const uint64_t* p) {
    return *reinterpret_cast<const __attribute__((address_space(1))) uint64_t*>(reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ u64x2_a8 gload16a8(const uint64_t* p) {
    return *reinterpret_cast<const __attribute__((address_space(1))) u64x2_a8*>(reinterpret_cast<uintptr_t>(p));
}
template <int PAD>
struct MsgView {
    const uint32_t* woff;   // LDS: word offset of segment s in the payload, s <= count
    __device__ __forceinline__ uint32_t wo(uint32_t s) const {
        return PAD ? *reinterpret_cast<const uint32_t*>(msg_pad(const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(woff)), s))
                   : woff[s];
    }
    __device__ __forceinline__ uint64_t ba(uint32_t s) const {
        return PAD ? *reinterpret_cast<const uint64_t*>(
                         msg_pad(const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(woff)), 128 + 2 * s))
                   : base[s];
    }
    const uint64_t* base;   // device address of segment s (LDS, tiled pass)
    uint32_t count;         // segments (>= 1)
    uint32_t hw;            // header words
};

// Word q of the framed stream (q < total words). `s` is a segment hint: the segment
// holding the previous payload word (advanced forward, so a lane's consecutive words
// cost one search).
template <int PAD>
__device__ __forceinline__ uint64_t msg_word(const MsgView<PAD>& m, uint32_t q, uint32_t& s) {
    if (q < m.hw) {  // toBytes 2147-2163: u32 j = count - 1 (j = 0), size_{j-1} (1 <= j <= count), pad
        uint32_t v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t j = 2 * q + h;
            v[h] = j == 0 ? m.count - 1 : (j <= m.count ? m.wo(j) - m.wo(j - 1) : 0u);
        }
        return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
    }
    const uint32_t p = q - m.hw;
    if (s >= m.count || p < m.wo(s)) {  // (re)search: largest s with woff[s] <= p, non-empty
        uint32_t lo = 0, hi = m.count;  // woff[lo] <= p < woff[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (m.wo(mid) <= p) lo = mid;
            else hi = mid;
        }
        s = lo;
    }
    while (p >= m.wo(s + 1)) ++s;  // skip to the segment holding p (empty ones included)
    return gload8(reinterpret_cast<const uint64_t*>(m.ba(s) + 8ull * (p - m.wo(s))));
}

// Stage framed words [tb, tb + tw) (tw <= 512) into the row layout. Lane l gathers
// words tb + l + 64j: consecutive lanes read consecutive words (coalesced within a
// segment), and all 8 addresses are formed before any load is issued, so the 8
// loads are in flight together.
template <int PAD>
__device__ __forceinline__ void msg_stage(const MsgView<PAD>& m, uint32_t tb, uint32_t tw, uint32_t lane, uint32_t& hint,
                                          uint8_t* lds) {
    const uint64_t* src[8];
    uint64_t hv[8];
    uint32_t wlo = 1, whi = 0;  // cached segment window [wlo, whi) of payload words (empty)
    uint64_t wbase = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t i = lane + 64 * j;
        src[j] = nullptr;
        hv[j] = 0;
        if (i < tw) {
            const uint32_t q = tb + i;
            if (q < m.hw) {
                hv[j] = msg_word(m, q, hint);  // header word (no load)
            } else {
                const uint32_t p = q - m.hw;
                if (p < wlo || p >= whi) {  // leave the cached segment window: search, then cache
                    if (hint >= m.count || p < m.wo(hint)) {
                        uint32_t lo = 0, hi = m.count;
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (m.wo(mid) <= p) lo = mid;
                            else hi = mid;
                        }
                        hint = lo;
                    }
                    while (p >= m.wo(hint + 1)) ++hint;
                    wlo = m.wo(hint);
                    whi = m.wo(hint + 1);
                    wbase = m.ba(hint);
                }
                src[j] = reinterpret_cast<const uint64_t*>(wbase + 8ull * (p - wlo));
            }
        }
    }
    uint64_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = src[j] ? gload8(src[j]) : hv[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t i = lane + 64 * j;
        if (i < tw) *reinterpret_cast<uint64_t*>(lds + (i >> 3) * kEncRow + (i & 7) * 8) = x[j];
    }
}

// One-tile staging by word pairs: lane l gathers framed words 2l + 128j and 2l + 1 + 128j with
// one 16-B load when both lie in one segment (all but the segments' edges and the header), else
// word by word, and writes the pair to its row with one 16-B LDS store: half the load
// instructions of msg_stage's word-per-load gather. All addresses first, then every load, then
// the LDS stores, so the loads are in flight together. Segments are found through a per-word
// map, seg_of[p] (u8, payload word p -> its segment + 1), built once per message in the tile's
// row data (zeroed, each non-empty segment marks its first word, a forward fill by lane and a
// wave max-scan: segment starts increase with the index): one LDS byte read per word and no
// search loop (a per-lane search with a cached window measured 2.37-2.38 ms on the framing leg
// against 2.16 ms, same box). The map is read only while the addresses are formed, before any
// staged word is written.
__device__ __forceinline__ void msg_stage_pairs_map(const MsgView<1>& m, uint32_t tw, uint32_t lane, uint8_t* lds,
                                                    uint32_t my_woff, bool my_mark) {
    auto map_at = [&](uint32_t p) -> uint8_t* { return lds + (p >> 6) * kEncRow + (p & 63); };
    const bool one = m.count == 1;  // wave-uniform: a one-segment message needs no map
    if (!one) {
    *reinterpret_cast<uint64_t*>(lds + (lane >> 3) * kEncRow + 8 * (lane & 7)) = 0;  // words 8l .. 8l+7
    wave_lds_sync();
    if (my_mark) *map_at(my_woff) = (uint8_t)(lane + 1);
    wave_lds_sync();
    uint64_t v = *reinterpret_cast<const uint64_t*>(lds + (lane >> 3) * kEncRow + 8 * (lane & 7));
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // forward fill inside the lane's 8 words
        const uint32_t b = (uint32_t)(v >> (8 * k)) & 0xFFu;
        run = b ? b : run;
        v = (v & ~(0xFFull << (8 * k))) | ((uint64_t)run << (8 * k));
    }
    const uint32_t before = wave_prev_lane(wave_incl_max(run, lane), 0u);  // marks increase with p
    uint64_t fill = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t b = (uint32_t)(v >> (8 * k)) & 0xFFu;
        fill |= (uint64_t)(b ? b : before) << (8 * k);
    }
    *reinterpret_cast<uint64_t*>(lds + (lane >> 3) * kEncRow + 8 * (lane & 7)) = fill;
    wave_lds_sync();
    }

    const uint64_t* pa[4];
    const uint64_t* pb[4];
    uint64_t ha[4], hb[4];
    bool pair[4];
    uint32_t hh = 0;
    auto addr = [&](uint32_t p, uint32_t sg) {  // payload word p in segment sg
        return reinterpret_cast<const uint64_t*>(m.ba(sg) + 8ull * (p - m.wo(sg)));
    };
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = 2 * lane + 128 * j;
        pa[j] = pb[j] = nullptr;
        ha[j] = hb[j] = 0;
        pair[j] = false;
        if (i < tw) {
            const bool two = i + 1 < tw;
            // header words (at most 33) only in the first 128-word block
            const bool hda = j == 0 && i < m.hw, hdb = j == 0 && i + 1 < m.hw;
            uint32_t sa = 0;
            if (hda) {
                ha[j] = msg_word(m, i, hh);
            } else {
                const uint32_t p = i - m.hw;
                sa = one ? 0u : *map_at(p) - 1u;
                pa[j] = addr(p, sa);
            }
            if (two) {
                if (hdb) {
                    hb[j] = msg_word(m, i + 1, hh);
                } else {
                    const uint32_t p = i + 1 - m.hw;
                    const uint32_t sb = one ? 0u : *map_at(p) - 1u;
                    if (!hda && sb == sa) pair[j] = true;
                    else pb[j] = addr(p, sb);
                }
            }
        }
    }
    uint64_t xa[4], xb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (pair[j]) {
            const u64x2_a8 w = gload16a8(pa[j]);
            xa[j] = w.x;
            xb[j] = w.y;
        } else {
            xa[j] = pa[j] ? gload8(pa[j]) : ha[j];
            xb[j] = pb[j] ? gload8(pb[j]) : hb[j];
        }
    }
    wave_lds_sync();  // every lane has read the map
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = 2 * lane + 128 * j;
        uint8_t* const d = lds + (i >> 3) * kEncRow + (i & 7) * 8;
        if (i + 1 < tw) *reinterpret_cast<u32x4*>(d) = u32x4{(uint32_t)xa[j], (uint32_t)(xa[j] >> 32),
                                                              (uint32_t)xb[j], (uint32_t)(xb[j] >> 32)};
        else if (i < tw) *reinterpret_cast<uint64_t*>(d) = xa[j];
    }
}

// One message of at most 64 segments and one framed tile (<= 512 words), a wave: lane s loads
// segment s's length and address (two coalesced loads), a wave scan gives the word offsets, and
// offsets and addresses go to the row pads (MsgView<1>); then the pair gather and encode_tile.
// Anything else (more segments or words, and the argument checks that come with them) is
// marked for the tiled pass (kStNeedFull), which applies toBytes' checks in the reference order.
// The message once its table is in registers: c_in segments (uniform), lane s holding segment
// s's length and address. (A persistent form that loaded the next message's table while this
// one was coded ran at 91 VGPRs, 5 waves/SIMD, and took 2.48-2.50 ms on the framing leg against
// 2.15-2.16 ms for this one at 7: DESIGN.md §2.5.)
template <bool WRITE>
__device__ __forceinline__ void encode_message_tile1_body(uint32_t msg, uint32_t lane, const uint64_t* lut,
                                                          uint8_t* lds, uint32_t c_in, uint64_t len, uint64_t ptr,
                                                          uint64_t ob, uint64_t cap, uint8_t* __restrict__ out,
                                                          uint64_t* __restrict__ out_len,
                                                          int32_t* __restrict__ status) {
    const uint32_t count = c_in == 0 ? 1u : c_in;  // toBytes 2128-2130: at least one (empty) segment
    // segments are whole words at 8-B aligned addresses (a MessageBuilder's always are); any
    // segment of more than a tile sends the message to the tiled pass before the u32 sum
    const bool odd = (len & 7) != 0 || (ptr & 7) != 0;
    const bool big = (len >> 3) > kEncMaxWords;
    if (count > kMsgOneSegs || __builtin_amdgcn_ballot_w64(odd || big) != 0) {
        if (lane == 0) status[msg] = kStNeedFull;  // the tiled pass reports ST_ARG / codes it
        return;
    }
    const uint32_t wl = (uint32_t)(len >> 3);
    const uint32_t incl = wave_incl_sum(wl, lane);
    const uint32_t payload = readlane(incl, 63);
    const uint32_t hw = (1 + count + ((count & 1) ? 0 : 1)) / 2;  // toBytes 2135-2137, in words
    const uint32_t words = hw + payload;
    if (words > kEncMaxWords) {
        if (lane == 0) status[msg] = kStNeedFull;
        return;
    }
    // Segments laid end to end (each starts where the previous one ends, as a MessageBuilder's
    // arena or a pool of one message's segments has them): the payload is one run, staged as
    // encode_kernel stages a unit (coalesced 16-B loads), after the segment table's words, which
    // lanes < hw compute from the segment lengths (toBytes 2147-2163). No map, no per-word search.
    const uint64_t nptr = shfl_u64(ptr, min(lane + 1, 63u));
    if (__builtin_amdgcn_ballot_w64(lane + 1 < count && ptr + len != nptr) == 0) {
        const uint32_t ja = 2 * lane, jb = 2 * lane + 1;  // u32 entries of header word `lane`
        const uint32_t sa = (uint32_t)__shfl((int)wl, (int)(ja == 0 ? 0u : min(ja - 1, 63u)), kWave);
        const uint32_t sb = (uint32_t)__shfl((int)wl, (int)min(jb - 1, 63u), kWave);
        const uint32_t ha = ja == 0 ? count - 1 : (ja <= count ? sa : 0u);
        const uint32_t hb = jb <= count ? sb : 0u;
        const uint8_t* const src = reinterpret_cast<const uint8_t*>(shfl_u64(ptr, 0));
        uint4 v[5];
        if (payload) encode_load(v, src, payload, lane);
        if (lane < hw) *reinterpret_cast<uint64_t*>(lds + (lane >> 3) * kEncRow + (lane & 7) * 8) =
            (uint64_t)ha | ((uint64_t)hb << 32);
        if (payload) encode_put_at(lds, v, (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15), payload, lane, hw);
        wave_lds_sync();
        uint32_t cz = 0, cf = 0;
        const uint32_t P = encode_tile<WRITE, true>(lds, lut, lane, words, 0, cz, cf, words, words, out + ob, cap);
        if (lane == 0) {
            out_len[msg] = P;
            status[msg] = (WRITE && (uint64_t)P > cap) ? ST_SPACE : ST_OK;
        }
        return;
    }
    if (lane < count) {
        *reinterpret_cast<uint32_t*>(msg_pad(lds, lane)) = incl - wl;
        *reinterpret_cast<uint64_t*>(msg_pad(lds, 128 + 2 * lane)) = ptr;
    }
    if (lane == 63) *reinterpret_cast<uint32_t*>(msg_pad(lds, count)) = payload;  // woff[count]
    wave_lds_sync();
    const MsgView<1> m{reinterpret_cast<const uint32_t*>(lds), nullptr, count, hw};
    msg_stage_pairs_map(m, words, lane, lds, incl - wl, lane < count && wl != 0);
    wave_lds_sync();
    uint32_t cz = 0, cf = 0;
    const uint32_t P = encode_tile<WRITE, true>(lds, lut, lane, words, 0, cz, cf, words, words, out + ob, cap);
    if (lane == 0) {
        out_len[msg] = P;
        status[msg] = (WRITE && (uint64_t)P > cap) ? ST_SPACE : ST_OK;
    }
}

// One message (see encode_message_kernel); lds / woff / base are the wave's slices.
template <bool WRITE, bool TILED>
__device__ __forceinline__ void encode_message_one(uint32_t msg, uint32_t lane, const uint64_t* lut, uint8_t* lds,
                                                   uint32_t* woff, uint64_t* base,
                                                   const uint64_t* __restrict__ seg_ptr,
                                                   const uint64_t* __restrict__ seg_len,
                                                   const uint32_t* __restrict__ seg_first,
                                                   const uint32_t* __restrict__ seg_count, uint8_t* __restrict__ out,
                                                   const uint64_t* __restrict__ out_off,
                                                   const uint64_t* __restrict__ out_cap,
                                                   uint64_t* __restrict__ out_len, int32_t* __restrict__ status) {

    // ---- segment table: lane l takes segments 8l .. 8l+7 ------------------------------
    const uint32_t c_in = seg_count[msg];
    const uint32_t first = seg_first[msg];
    const uint32_t count = c_in == 0 ? 1u : c_in;  // toBytes 2128-2130: at least one (empty) segment
    if (count > kMsgMaxSegs) {
        if (lane == 0) { out_len[msg] = 0; status[msg] = ST_ARG; }
        return;
    }
    static_assert(TILED, "one-tile messages: encode_message_tile1_body");
    auto wput = [&](uint32_t s, uint32_t v) { woff[s] = v; };
    uint32_t wsum = 0;
    bool bad = false;
    uint32_t wl[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t s = 8 * lane + t;
        wl[t] = 0;
        if (s < count) {
            uint64_t len = 0, ptr = 0;
            if (c_in) {
                len = seg_len[first + s];
                ptr = seg_ptr[first + s];
            }
            // segments are whole words at 8-B aligned addresses (a MessageBuilder's always are)
            bad |= (len & 7) != 0 || (ptr & 7) != 0 || (len >> 3) > 0xFFFFFFFFull;
            wl[t] = (uint32_t)(len >> 3);
            base[s] = ptr;
            wsum += wl[t];
        }
    }
    const uint32_t incl = wave_incl_sum(wsum, lane);
    uint32_t acc = incl - wsum;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t s = 8 * lane + t;
        if (s < count) wput(s, acc);
        acc += wl[t];
    }
    const uint32_t payload = readlane(incl, 63);
    if (lane == 63) wput(count, payload);
    const uint32_t hw = (1 + count + ((count & 1) ? 0 : 1)) / 2;  // toBytes 2135-2137, in words
    const uint64_t words64 = (uint64_t)hw + payload;
    if (__builtin_amdgcn_ballot_w64(bad) != 0 || words64 > 0xFFFFF000ull) {
        if (lane == 0) { out_len[msg] = 0; status[msg] = ST_ARG; }
        return;
    }
    const uint32_t words = (uint32_t)words64;
    wave_lds_sync();
    const MsgView<0> m{woff, base, count, hw};
    uint64_t ob = 0, cap = 0;
    if (WRITE) {
        ob = out_off[msg];
        cap = out_cap[msg];
    }

    // ---- tiles, as in encode_tiled_kernel ------------------------------------------------
    uint32_t cz = 0, cf = 0, hint = 0xFFFFFFFFu;
    uint64_t pos = 0;
    bool fits = true;
    for (uint32_t tb = 0; tb < words; tb += kEncMaxWords) {
        // lane-derived addresses are recomputed per tile, not held across the loops in
        // registers (loop-invariant hoisting had this kernel at 140 VGPRs)
        uint32_t lane_u = lane;
        asm volatile("" : "+v"(lane_u));
        const uint32_t tw = min(kEncMaxWords, words - tb);
        const uint32_t te = tb + tw;
        uint32_t nbz = words, nbf = words;
        if (te < words) {  // first Z / F break in the 256 words after the tile
            const uint32_t la = min(256u, words - te);
            uint32_t fz = la, ff = la, h2 = 0xFFFFFFFFu;
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t i = 4 * lane + t;
                if (i < la) {
                    const uint32_t tg = nonzero_tag(msg_word(m, te + i, h2));
                    if (tg != 0 && fz == la) fz = i;
                    if (tg != 0xFF && ff == la) ff = i;
                }
            }
            const uint32_t bz = wave_min(fz), bf = wave_min(ff);
            nbz = bz < la ? te + bz : (la == 256u ? te + 256u : words);
            nbf = bf < la ? te + bf : (la == 256u ? te + 256u : words);
        }
        wave_lds_sync();  // the previous tile's write-back read the slice
        msg_stage(m, tb, tw, lane, hint, lds);
        wave_lds_sync();
        const uint64_t room = (WRITE && fits && pos <= cap) ? cap - pos : 0;
        const uint32_t Pt = encode_tile<WRITE, false>(lds, lut, lane, tw, tb, cz, cf, nbz, nbf, out + ob + pos,
                                                      room);
        if ((uint64_t)Pt > room) fits = false;
        pos += Pt;
    }
    if (lane == 0) {
        out_len[msg] = pos;
        status[msg] = (WRITE && !fits) ? ST_SPACE : ST_OK;
    }
}

// TILED = false: every message, two per wave; one framed tile (<= 512 words) of at most 64
// segments is encoded here (encode_message_tile1_body: segments end to end staged as one run,
// else offsets and addresses in the tile's row pads and the pair gather), other
// messages are marked for TILED = true, which keeps the offsets and addresses in LDS arrays,
// applies the argument checks and walks the tiles.
// The multi-tile pass strides over the batch with a small grid, 64 statuses per load.
template <bool WRITE, bool TILED>
__global__ __launch_bounds__(kBlock) void encode_message_kernel(const uint64_t* __restrict__ seg_ptr,
                                                                const uint64_t* __restrict__ seg_len,
                                                                const uint32_t* __restrict__ seg_first,
                                                                const uint32_t* __restrict__ seg_count, uint32_t n,
                                                                uint8_t* __restrict__ out,
                                                                const uint64_t* __restrict__ out_off,
                                                                const uint64_t* __restrict__ out_cap,
                                                                uint64_t* __restrict__ out_len,
                                                                int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kEncLds];
    __shared__ uint32_t woff_all[TILED ? kWavesPerBlock * (kMsgMaxSegs + 1) : 1];
    __shared__ uint64_t base_all[TILED ? kWavesPerBlock * kMsgMaxSegs : 1];
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (WRITE) {
        lut[threadIdx.x] = compact_selector(threadIdx.x);
        __syncthreads();
    }
    uint8_t* const lds = smem + wave * kEncLds;
    uint32_t* const woff = woff_all + wave * (kMsgMaxSegs + 1);
    uint64_t* const base = TILED ? base_all + wave * kMsgMaxSegs : nullptr;
    if (!TILED) {
        // two messages per wave: both segment tables are loaded before the first is coded, so
        // the second's dependent load level (count / first -> lengths / addresses -> data) is
        // hidden behind the first's coding
        const uint32_t m0 = 2 * (blockIdx.x * kWavesPerBlock + wave), m1 = m0 + 1;
        if (m0 >= n) return;
        const bool two = m1 < n;
        const uint32_t c0 = seg_count[m0], f0 = seg_first[m0];
        const uint32_t c1 = two ? seg_count[m1] : 0u, f1 = two ? seg_first[m1] : 0u;
        uint64_t len0 = 0, ptr0 = 0, len1 = 0, ptr1 = 0;
        if (c0 && c0 <= kMsgOneSegs && lane < c0) {
            len0 = seg_len[f0 + lane];
            ptr0 = seg_ptr[f0 + lane];
        }
        if (two && c1 && c1 <= kMsgOneSegs && lane < c1) {
            len1 = seg_len[f1 + lane];
            ptr1 = seg_ptr[f1 + lane];
        }
        uint64_t ob0 = 0, cap0 = 0, ob1 = 0, cap1 = 0;
        if (WRITE) {
            ob0 = out_off[m0];
            cap0 = out_cap[m0];
            if (two) {
                ob1 = out_off[m1];
                cap1 = out_cap[m1];
            }
        }
        encode_message_tile1_body<WRITE>(m0, lane, lut, lds, c0, len0, ptr0, ob0, cap0, out, out_len, status);
        if (two) {
            wave_lds_sync();  // m0's write-back read the slice
            encode_message_tile1_body<WRITE>(m1, lane, lut, lds, c1, len1, ptr1, ob1, cap1, out, out_len, status);
        }
        return;
    }
    const uint32_t stride = gridDim.x * kWavesPerBlock * kWave;
    for (uint32_t ubase = (blockIdx.x * kWavesPerBlock + wave) * kWave; ubase < n; ubase += stride) {
        const uint32_t u = ubase + lane;
        uint64_t todo = __ballot(u < n && status[u] == kStNeedFull);
        while (todo) {
            const uint32_t msg = ubase + (uint32_t)__builtin_ctzll(todo);
            todo &= todo - 1;
            encode_message_one<WRITE, true>(msg, lane, lut, lds, woff, base, seg_ptr, seg_len, seg_first, seg_count,
                                            out, out_off, out_cap, out_len, status);
        }
    }
}

// ---------------------------------------------------------------------------
// Message.init on device (message.zig:341-394): the segment table of each framed
// message, lane per message. seg_off / seg_len get max_segs entries per message
// (row i at i * max_segs; segments past max_segs are counted, not listed).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void message_init_kernel(const uint8_t* __restrict__ in,
                                                              const uint64_t* __restrict__ in_off,
                                                              const uint64_t* __restrict__ in_len, uint32_t n,
                                                              uint32_t max_segs, uint32_t* __restrict__ seg_count,
                                                              uint64_t* __restrict__ seg_off,
                                                              uint64_t* __restrict__ seg_len,
                                                              int32_t* __restrict__ status) {
    const uint32_t msg = blockIdx.x * kBlock + threadIdx.x;
    if (msg >= n) return;
    const uint8_t* const d = in + in_off[msg];
    const uint64_t len = in_len[msg];
    auto u32at = [&](uint64_t o) {
        return (uint32_t)d[o] | ((uint32_t)d[o + 1] << 8) | ((uint32_t)d[o + 2] << 16) | ((uint32_t)d[o + 3] << 24);
    };
    int32_t st = ST_OK;
    uint64_t count = 0;
    if (len < 4) {
        st = ST_EOS;  // :343 readInt
    } else {
        const uint32_t m1 = u32at(0);
        if (m1 == 0xFFFFFFFFu) st = ST_SEGCOUNT;  // :346
        else if ((uint64_t)m1 + 1 > kMsgMaxSegs) st = ST_SEGLIMIT;  // :348
        else {
            count = (uint64_t)m1 + 1;
            const uint64_t header = 4 * (1 + count + ((count & 1) ? 0 : 1));
            if (header > len) st = ST_TRUNC;  // :353
            uint64_t o = header;
            for (uint64_t i = 0; st == ST_OK && i < count; ++i) {
                const uint64_t end = o + 8ull * u32at(4 + 4 * i);
                if (end > len) { st = ST_TRUNC; break; }  // :380
                if (i < max_segs) {
                    seg_off[(uint64_t)msg * max_segs + i] = o;
                    seg_len[(uint64_t)msg * max_segs + i] = end - o;
                }
                o = end;
            }
        }
    }
    seg_count[msg] = st == ST_OK ? (uint32_t)count : 0u;
    status[msg] = st;
}

// ---------------------------------------------------------------------------
// DECODE, lane per unit
// ---------------------------------------------------------------------------
// The record chain (tag -> record length) is inherently serial and speculative
// chunk walks couple with it too slowly on packed data, so each
// lane owns ONE unit and walks its chain exactly once, expanding every record as
// it is found. The lane keeps a sliding window of its packed bytes in registers:
// a 32-byte view (q0..q3) plus one 16-byte piece in flight (n0, n1). A CU holds
// thousands of units in flight, which hides the memory latency of each lane's
// dependent chain.

// View helpers take the window by value so the selects stay register selects
// (members selected through `this` were turned into an indexed alloca in LDS).
__device__ __forceinline__ uint32_t view_byte(uint64_t q0, uint64_t q1, uint64_t q2, uint64_t q3, uint32_t o) {
    uint64_t a = (o & 8) ? q1 : q0;  // o < 32
    uint64_t b = (o & 8) ? q3 : q2;
    uint64_t q = (o & 16) ? b : a;
    return (uint32_t)(q >> (8 * (o & 7))) & 0xFFu;
}
__device__ __forceinline__ uint64_t view_word8(uint64_t q0, uint64_t q1, uint64_t q2, uint64_t q3, uint32_t o) {
    // 8 bytes at view offset o, o <= 24
    uint32_t i = o >> 3;
    uint64_t lo = (i == 0) ? q0 : ((i == 1) ? q1 : q2);
    uint64_t hi = (i == 0) ? q1 : ((i == 1) ? q2 : q3);
    uint32_t sh = 8 * (o & 7);
    return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
}
__device__ __forceinline__ void load_piece(const uint8_t* base, uint32_t npieces, uint32_t idx, uint64_t& a,
                                           uint64_t& b) {
    if (idx < npieces) {
        uint4 v = *reinterpret_cast<const uint4*>(base + 16 * (uint64_t)idx);
        a = (uint64_t)v.x | ((uint64_t)v.y << 32);
        b = (uint64_t)v.z | ((uint64_t)v.w << 32);
    } else {
        a = 0;
        b = 0;
    }
}

template <bool WRITE, bool CK = false>
__global__ __launch_bounds__(kBlock) void decode_lane_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ in_off,
                                                             const uint64_t* __restrict__ in_len,
                                                             uint32_t n, uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off,
                                                             const uint64_t* __restrict__ out_cap,
                                                             uint64_t* __restrict__ out_len,
                                                             int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    if (WRITE) {
        lut[threadIdx.x] = expand_selector(threadIdx.x);
        __syncthreads();
    }
    const uint32_t unit = blockIdx.x * kBlock + threadIdx.x;
    if (unit >= n) return;
    if (CK && status[unit] != kStNeedFull) return;  // size-only fallback after decode_index_kernel<true>
    const uint8_t* src = in + in_off[unit];
    const uint64_t P = in_len[unit];
    uint64_t* dst = nullptr;
    uint64_t capw = 0;
    if (WRITE) {
        uint8_t* o = out + out_off[unit];
        if (P > 0 && (reinterpret_cast<uintptr_t>(o) & 7)) {  // an empty unit writes nothing
            out_len[unit] = 0;
            status[unit] = ST_ARG;
            return;
        }
        dst = reinterpret_cast<uint64_t*>(o);
        capw = out_cap[unit] >> 3;
    }
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    const uint64_t end64 = s + P;
    const uint8_t* base = src - s;
    const uint32_t npieces = (uint32_t)((end64 + 15) >> 4);
    // window: q0..q3 = pieces wb/16, wb/16+1; n0,n1 = piece wb/16+2 (in flight)
    uint64_t q0, q1, q2, q3, n0, n1;
    uint32_t wb = 0;
    load_piece(base, npieces, 0, q0, q1);
    load_piece(base, npieces, 1, q2, q3);
    load_piece(base, npieces, 2, n0, n1);
    auto ensure = [&](uint32_t p) {
        while (p - wb >= 16) {
            q0 = q2; q1 = q3; q2 = n0; q3 = n1;
            wb += 16;
            load_piece(base, npieces, (wb >> 4) + 2, n0, n1);
        }
    };
    uint64_t pos = s;
    uint64_t wo = 0;
    int32_t st = ST_OK;
    auto put = [&](uint64_t w) {
        if (WRITE && wo < capw) dst[wo] = w;
        ++wo;
    };
    while (pos < end64) {
        ensure((uint32_t)pos);
        const uint32_t o = (uint32_t)pos - wb;
        const uint32_t t = view_byte(q0, q1, q2, q3, o);
        if (t == 0x00) {  // message.zig:101-110
            if (pos + 2 > end64) { st = ST_EOF; break; }
            const uint32_t c = view_byte(q0, q1, q2, q3, o + 1);
            for (uint32_t k = 0; k <= c; ++k) put(0);
            pos += 2;
        } else if (t == 0xFF) {  // message.zig:112-128
            if (pos + 10 > end64) { st = ST_EOF; break; }
            const uint64_t w = view_word8(q0, q1, q2, q3, o + 1);
            const uint32_t c = view_byte(q0, q1, q2, q3, o + 9);
            if (pos + 10 + 8ULL * c > end64) { st = ST_EOF; break; }
            put(w);
            pos += 10;
            for (uint32_t k = 0; k < c; ++k) {
                ensure((uint32_t)pos);
                put(view_word8(q0, q1, q2, q3, (uint32_t)pos - wb));
                pos += 8;
            }
        } else {  // message.zig:131-141
            const uint32_t k = __popc(t);
            if (pos + 1 + k > end64) { st = ST_EOF; break; }
            if (WRITE) put(perm64(view_word8(q0, q1, q2, q3, o + 1), lut[t]));
            else put(0);
            pos += 1 + k;
        }
    }
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    const uint64_t U = 8 * wo;
    out_len[unit] = U;
    status[unit] = (WRITE && wo > capw) ? ST_SPACE : ST_OK;
}

// ---------------------------------------------------------------------------
// DECODE fallback, wave per unit (long units of the indexed decoder, marked units
// of the read-message passes; profiles/r01_decode_experiments.md)
// ---------------------------------------------------------------------------
// One wave owns one unit. The unit's packed bytes are processed in windows of
// up to kWvWin bytes (one window for units up to ~4.5 KiB packed), each staged
// in the wave's LDS slice with coalesced 16-B loads. Lane j owns the chunk
// [j*C, (j+1)*C) of the window and must find the true record chain through it
// (tag -> record length -> next tag, message.zig:152-191), which is serial:
//
//   walk A   every lane walks its chunk from the chunk start (a guess),
//            marking the tags it visits in a per-byte mark array (walk id 1);
//   walk B   every lane walks from the exit of its left neighbour's walk A
//            (the neighbour's guess of where the chain enters this chunk),
//            stopping as soon as it reaches a marked tag: from there the
//            chain is the marked walk's, so its exit is known (walk id 2);
//   rounds   lane j is verified when its entry equals lane j-1's exit and
//            lane j-1 is verified (lane 0 enters at 0, the window start is a
//            tag). Every lane whose entry disagrees re-walks from its
//            neighbour's exit, again stopping at the first marked tag. Each
//            round verifies at least the first disagreeing lane, so this ends
//            in <= 64 rounds; because chains from different entries couple
//            within a few records, 0-2 rounds are typical.
//   count    each lane sums the output words of its verified records; a wave
//            scan gives every lane its output word offset;
//   expand   each lane expands its records (v_perm_b32 scatter of the nonzero
//            bytes) and stores the words; zero runs and literal runs longer
//            than a few words are handed to the whole wave (coalesced).
//
// The window's exit (lane 63's verified exit) is the next window's start, so
// any unit size works; LDS-resident chunks keep every chain step an LDS read.
constexpr uint32_t kWvWaves = 4;                      // waves (units) per block
constexpr uint32_t kWvBlock = kWvWaves * kWave;
constexpr uint32_t kWvWin = 4608;                     // packed bytes per window (64 chunks x 72 B)
constexpr uint32_t kWvPk = kWvWin + 64;               // + 15 B alignment slack + 16 B overshoot + read slack
constexpr uint32_t kWvCmin = 32;                      // minimum chunk bytes per lane
constexpr uint32_t kWvStageK = (kWvPk / 16 + 63) / 64;
constexpr uint32_t kEOFX = 0xFFFFFFFFu;               // "the chain ran past the end of the input"
constexpr uint32_t kWvExtLane = 3;                    // longer literal runs are listed by the whole wave
constexpr uint32_t kWvList = 1024;                    // output words per expand pass (u16 list in the mark array)
constexpr uint32_t kPosMask = 0x1FFFu;                // list code: window position (< 8192)
constexpr uint32_t kLit = 0x2000u;                    // list code: literal word (identity selector)
constexpr uint32_t kZero = 0x8000u;                   // list code: zero word
constexpr uint32_t kZero2 = kZero | (kZero << 16);
static_assert(kWvList * 2 <= kWvWin, "list aliases the mark array");
static_assert(kWvWin + 16 + 2058 < 8192, "list codes hold window positions");
constexpr uint32_t kWvSlack = 16;                     // plausible entry offset into a chunk (records are <= 9 B)

__device__ __forceinline__ uint32_t wv_sel_exit(uint32_t m, uint32_t e1, uint32_t e2, uint32_t e3, uint32_t e4,
                                                uint32_t e5, uint32_t e6, uint32_t e7) {
    uint32_t r = e7;
    r = (m == 6) ? e6 : r;
    r = (m == 5) ? e5 : r;
    r = (m == 4) ? e4 : r;
    r = (m == 3) ? e3 : r;
    r = (m == 2) ? e2 : r;
    r = (m == 1) ? e1 : r;
    return r;
}

// Walk the chain from window position r to the first tag position >= cend,
// marking visited tags with id (id 0: no marks). Stops at a tag marked by an
// earlier walk and reports its id in hit (the caller maps it to that walk's
// exit). Returns kEOFX if a record runs past the input end (rem bytes).
__device__ __forceinline__ uint32_t wv_len(uint32_t t, uint32_t c) {  // record length for tag t
    const uint32_t zf = (t == 0u) | (t == 0xFFu);             // 00 -> 2, FF -> 10 + 8c, else 1 + popc
    return 1u + __popc(t) + zf + ((t == 0xFFu) ? 8u * c : 0u);
}

__device__ __forceinline__ uint32_t wv_walk(const uint8_t* pk, uint8_t* mk, uint32_t sh, uint32_t rem, uint32_t r,
                                            uint32_t cend, uint32_t id, uint32_t& hit) {
    uint32_t h = 0;
    bool go = r < cend;
    while (go) {  // body is branch-free: one loop exit
        uint32_t m = mk[r];
        uint32_t t = pk[sh + r];
        uint32_t c = pk[sh + r + 9];
        asm volatile("" : "+v"(m), "+v"(t), "+v"(c));  // issue the three LDS reads together, one wait
        const uint32_t len = wv_len(t, c);
        const bool coupled = m != 0;
        mk[r] = (uint8_t)(coupled ? m : id);  // unconditional: rewrites m where coupled or id == 0
        h = m;
        const uint32_t nr = (r + len > rem) ? kEOFX : r + len;
        r = coupled ? r : nr;
        go = !coupled && r < cend;
    }
    hit = h;
    return r;
}

// Unaligned 8-byte LDS read as two aligned ds_read_b64 and a branch-free funnel
// shift (a byte-aligned ds_read_b64 is legal on gfx950 but measured ~2x slower
// in the expand loop: the LDS splits it).
__device__ __forceinline__ uint64_t lds_u64_at(const uint8_t* base, uint32_t p) {
    const uint32_t a = p & ~7u;
    const uint64_t lo = *reinterpret_cast<const uint64_t*>(base + a);
    const uint64_t hi = *reinterpret_cast<const uint64_t*>(base + a + 8);
    const uint32_t s = (p & 7u) * 8u;
    return (lo >> s) | ((hi << 1) << (63u - s));
}
// Unaligned 8-byte global read (gfx950 unaligned-buffer-access: one global_load_dwordx2).
__device__ __forceinline__ uint64_t gload_u64_unaligned(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}


// A window of a unit's packed bytes staged in the wave's LDS slice: window byte r (unit
// byte X + r) at pk[sh + r] for r < nload. Records starting in [0, Pw) belong to the
// window; nload adds the <= 9 bytes such a record reaches past Pw.
struct WvWin {
    const uint8_t* g;  // unit byte X
    uint32_t sh;       // g & 15
    uint32_t rem;      // unit bytes from X on (clamped to 2^31 - 1)
    uint32_t Pw;       // window bytes
    uint32_t nload;    // staged bytes
};

// Stage window [X, X + kWvWin) of a unit of P packed bytes and clear its marks.
__device__ __forceinline__ WvWin wv_stage(uint8_t* pk, uint8_t* mk, const uint8_t* src, uint64_t P, uint64_t X,
                                          uint32_t lane) {
    WvWin w;
    const uint64_t rem64 = P - X;
    w.rem = rem64 > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)rem64;
    w.Pw = min(w.rem, kWvWin);
    w.nload = min(w.rem, w.Pw + 16);
    w.g = src + X;
    w.sh = (uint32_t)(reinterpret_cast<uintptr_t>(w.g) & 15);
    wave_lds_sync();
    stage_linear<kWvStageK>(pk, w.g - w.sh, (w.sh + w.nload + 15) >> 4, lane);
    for (uint32_t i = lane * 16; i < w.Pw; i += 16 * kWave) *reinterpret_cast<uint4*>(mk + i) = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
    return w;
}

// The record chain through a staged window whose first record starts at window byte d0
// (lane 0's entry, exact). Lane j owns the chunk [cs, ce); on return `ent` is the verified
// record start where the chain enters it, and the result is the window's exit: the first
// record start at or past Pw (window-relative), or kEOFX when a record runs past the
// unit's end (walks A and B and the verification rounds: see above).
__device__ __forceinline__ uint32_t wv_resolve(const uint8_t* pk, uint8_t* mk, const WvWin& w, uint32_t d0,
                                               uint32_t lane, uint32_t& ent, uint32_t& cs, uint32_t& ce) {
    const uint32_t C = max(kWvCmin, (w.Pw + 63) >> 6);
    cs = min(lane * C, w.Pw);
    ce = min(cs + C, w.Pw);

    // ---- walk A: lane 0 from d0, every other lane from its chunk start (a guess) -----
    const uint32_t a0 = lane == 0 ? d0 : cs;
    uint32_t hit;
    const uint32_t e1 = wv_walk(pk, mk, w.sh, w.rem, a0, ce, 1, hit);
    uint32_t e2 = 0, e3 = 0, e4 = 0, e5 = 0, e6 = 0, e7 = 0;

    // ---- walk B: enter where the left neighbour's walk A left off ---------------------
    // An entry far past the chunk start (a misread FF run, or a misread record running
    // past the input end) would only pass through; keep walk A's guess.
    ent = __shfl_up(e1, 1, kWave);
    if (lane == 0) ent = d0;
    else if (ent > cs + kWvSlack) ent = cs;
    uint32_t ex = e1;
    if (ent != a0) {
        ex = wv_walk(pk, mk, w.sh, w.rem, ent, ce, 2, hit);
        if (hit) ex = wv_sel_exit(hit, e1, e2, e3, e4, e5, e6, e7);
        e2 = ex;
    }

    // ---- verification rounds ------------------------------------------------------------
    // Lanes before the first disagreeing lane f are verified. A disagreeing lane re-walks
    // from its neighbour's exit when that neighbour is verified (lane f), or when the
    // neighbour agrees with ITS neighbour this round and the exit is a plausible entry
    // (<= kWvSlack into the chunk): far or EOF exits adopted from an unverified neighbour
    // would otherwise ripple one lane per round.
    uint32_t nid = 3;
    for (;;) {
        uint32_t prev = __shfl_up(ex, 1, kWave);
        if (lane == 0) prev = d0;
        const bool bad = ent != prev;
        const uint64_t bm = __ballot(bad);
        if (!bm) break;
        const uint32_t f = (uint32_t)__builtin_ctzll(bm);
        const bool left_bad = lane > 0 && ((bm >> (lane - 1)) & 1);
        if (bad && (lane == f || (!left_bad && prev <= cs + kWvSlack))) {
            ent = prev;
            const uint32_t id = nid <= 7 ? nid : 0;
            ex = wv_walk(pk, mk, w.sh, w.rem, ent, ce, id, hit);
            if (hit) ex = wv_sel_exit(hit, e1, e2, e3, e4, e5, e6, e7);
            e3 = (id == 3) ? ex : e3;
            e4 = (id == 4) ? ex : e4;
            e5 = (id == 5) ? ex : e5;
            e6 = (id == 6) ? ex : e6;
            e7 = (id == 7) ? ex : e7;
            ++nid;
        }
    }
    return readlane(ex, kWave - 1);
}

// Output words of a lane's verified records [ent, ce).
__device__ __forceinline__ uint32_t wv_count(const uint8_t* pk, uint32_t sh, uint32_t ent, uint32_t ce) {
    uint32_t words = 0;
    for (uint32_t r = ent; r < ce;) {
        uint32_t t = pk[sh + r];
        uint32_t b1 = pk[sh + r + 1];
        uint32_t c9 = pk[sh + r + 9];
        asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));
        words += 1u + ((t == 0u) ? b1 : 0u) + ((t == 0xFFu) ? c9 : 0u);
        r += wv_len(t, c9);
    }
    return words;
}

// Expand the window's verified records into o[0 .. total): lane records produce words
// [wbeg, wend). Passes of kWvList output words:
//   list:   each lane walks its verified records once more and writes, for every output
//           word of the pass that its records produce, a 16-bit source code into a list
//           in LDS (the mark array, dead by now): code = q (window position of a tag;
//           word = perm(bytes q+1..q+8, lut[byte q])) or kLit | (s - 1) (literal word at
//           bytes s..s+7); zero-run words keep the kZero code the list is reset to;
//   expand: lane i turns list entry i into its word and stores it, so every store
//           instruction writes 64 consecutive output words (512 B).
__device__ __forceinline__ void wv_expand(const uint8_t* pk, uint8_t* mk, const uint64_t* lut, const WvWin& w,
                                          uint32_t ent, uint32_t ce, uint32_t wbeg, uint32_t wend, uint32_t total,
                                          uint64_t* o, uint32_t lane) {
    const uint32_t sh = w.sh;
    uint16_t* const list = reinterpret_cast<uint16_t*>(mk);
    for (uint32_t W0 = 0; W0 < total; W0 += kWvList) {
        const uint32_t W1 = min(total, W0 + kWvList);
        wave_lds_sync();
        for (uint32_t i = lane * 8; i < kWvList; i += 8 * kWave)
            *reinterpret_cast<uint4*>(list + i) = make_uint4(kZero2, kZero2, kZero2, kZero2);
        wave_lds_sync();
        uint32_t pn = 0, ps = 0, pw = 0;  // long literal run handed to the wave
        if (wbeg < W1 && wend > W0) {
            uint32_t wo = wbeg;
            for (uint32_t r = ent; r < ce && wo < W1;) {
                uint32_t t = pk[sh + r];
                uint32_t b1 = pk[sh + r + 1];
                uint32_t c9 = pk[sh + r + 9];
                asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));
                const bool z = t == 0, f = t == 0xFFu;
                if (!z && wo >= W0) list[wo - W0] = (uint16_t)r;
                if (f && c9) {  // literal words r+10 .. r+10+8c
                    if (c9 <= kWvExtLane || pn != 0) {  // one long run per lane goes to the wave
                        for (uint32_t i = 0; i < c9; ++i) {
                            const uint32_t wi = wo + 1 + i;
                            if (wi >= W0 && wi < W1) list[wi - W0] = (uint16_t)(kLit | (r + 9 + 8 * i));
                        }
                    } else {
                        pn = c9;
                        ps = r + 9;
                        pw = wo + 1;
                    }
                }
                wo += 1u + (z ? b1 : 0u) + (f ? c9 : 0u);
                r += wv_len(t, c9);
            }
        }
        uint64_t pm = __ballot(pn != 0);
        while (pm) {  // long literal runs: the whole wave fills their entries
            const uint32_t l = (uint32_t)__builtin_ctzll(pm);
            pm &= pm - 1;
            const uint32_t nn = readlane(pn, l), ss = readlane(ps, l), ww = readlane(pw, l);
            for (uint32_t i = lane; i < nn; i += kWave) {
                const uint32_t wi = ww + i;
                if (wi >= W0 && wi < W1) list[wi - W0] = (uint16_t)(kLit | (ss + 8 * i));
            }
        }
        wave_lds_sync();
        for (uint32_t i = W0 + lane; i < W1; i += kWave) {
            const uint32_t code = list[i - W0];
            const uint32_t q = code & kPosMask;
            const bool lit = (code & kLit) != 0;
            uint64_t word = 0;
            if (!(code & kZero)) {
                if (!lit || q + 9 <= w.nload) {  // a tag's bytes are always staged
                    const uint32_t t = lit ? 0xFFu : pk[sh + q];
                    word = perm64(lds_u64_at(pk, sh + q + 1), lut[t]);
                } else {  // literal word past the staged bytes (long FF run), inside the input
                    word = gload_u64_unaligned(w.g + q + 1);
                }
            }
            __builtin_nontemporal_store(word, o + i);  // streaming output (as the fill pass)
        }
    }
}

// SEL: kWvMarked the units a first pass marked kStNeedFull (the read-message passes, the words
// decoder's units stopped at their capacity; q, when given, counts them: 0 returns at once);
// kWvLong the long units the window table could not hold (the serial list that
// long_windows_kernel fills), one after another.
constexpr int kWvMarked = 1, kWvLong = 2;

template <int SEL>
__global__ __launch_bounds__(kWvBlock) void decode_wave_kernel(const uint8_t* __restrict__ in,
                                                               const uint64_t* __restrict__ in_off,
                                                               const uint64_t* __restrict__ in_len, uint32_t n,
                                                               uint8_t* __restrict__ out,
                                                               const uint64_t* __restrict__ out_off,
                                                               const uint64_t* __restrict__ out_cap,
                                                               uint64_t* __restrict__ out_len,
                                                               int32_t* __restrict__ status, uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint8_t pk_all[kWvWaves * kWvPk];
    __shared__ __attribute__((aligned(16))) uint8_t mk_all[kWvWaves * kWvWin];
    __shared__ uint64_t lut[256];  // tag -> v_perm selector that scatters the packed bytes (FF: identity, 00: zero)
    constexpr bool CK = SEL == kWvMarked;
    if (CK && q && *q == 0) return;  // kWvMarked with a count of marked units: none
    const bool QD = SEL == kWvLong;
    if (QD && q[5] == 0) return;  // no serial units (block-uniform)
    lut[threadIdx.x] = expand_selector(threadIdx.x);
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* pk = pk_all + wave * kWvPk;
    uint8_t* mk = mk_all + wave * kWvWin;
    // CK: a first pass ran; this kernel takes only the units it marked kStNeedFull, with a
    // small grid striding over the batch (64 statuses per load). QD: the serial list, a
    // wave per entry striding over it (no shared atomic cursor: contended takes serialise).
    const uint32_t* const serial = q + serial_off(n);
    const uint32_t nq = QD ? q[5] : n;
    const uint32_t stride = QD ? gridDim.x * kWvWaves : gridDim.x * kWvWaves * kWave;
    for (uint32_t ubase = QD ? blockIdx.x * kWvWaves + wave : (blockIdx.x * kWvWaves + wave) * kWave; ubase < nq;
         ubase += stride) {
    uint64_t todo = 1;
    if (CK) {
        const uint32_t u = ubase + lane;
        todo = __ballot(u < n && status[u] == kStNeedFull);
    }
    while (todo) {  // wave-uniform
    const uint32_t unit = CK ? ubase + (uint32_t)__builtin_ctzll(todo) : __builtin_amdgcn_readfirstlane(serial[ubase]);
    todo &= todo - 1;
    const uint8_t* src = in + in_off[unit];
    const uint64_t P = in_len[unit];
    uint8_t* dstb = out + out_off[unit];
    const uint64_t capw = out_cap[unit] >> 3;
    if (reinterpret_cast<uintptr_t>(dstb) & 7) {
        if (lane == 0) {
            out_len[unit] = 0;
            status[unit] = ST_ARG;
        }
        continue;
    }
    uint64_t* const dst = reinterpret_cast<uint64_t*>(dstb);

    uint64_t X = 0;   // packed position of the current window (always a tag)
    uint64_t Wb = 0;  // output words before the current window
    int32_t st = ST_OK;
    bool fits = true;
    if (QD) {
        // a counting walk first (the serial units are the rare ones the window table
        // cannot hold): a truncated or oversized unit writes nothing, as unpackPacked
        // returns its error before any output (message.zig:88-145)
        while (X < P) {
            const WvWin w = wv_stage(pk, mk, src, P, X, lane);
            uint32_t ent, cs, ce;
            const uint32_t xw = wv_resolve(pk, mk, w, 0, lane, ent, cs, ce);
            if (xw == kEOFX) {
                st = ST_EOF;
                break;
            }
            const uint32_t words = wv_count(pk, w.sh, ent, ce);
            Wb += readlane(wave_incl_sum(words, lane), kWave - 1);
            X += xw;
        }
        if (st != ST_OK || Wb > capw) {
            if (lane == 0) {
                out_len[unit] = st == ST_OK ? 8 * Wb : 0;
                status[unit] = st != ST_OK ? st : ST_SPACE;
            }
            continue;
        }
        X = 0;
        Wb = 0;
    }
    while (X < P) {
        const WvWin w = wv_stage(pk, mk, src, P, X, lane);
        uint32_t ent, cs, ce;
        const uint32_t xw = wv_resolve(pk, mk, w, 0, lane, ent, cs, ce);
        if (xw == kEOFX) {
            st = ST_EOF;
            break;
        }
        const uint32_t words = wv_count(pk, w.sh, ent, ce);
        const uint32_t incl = wave_incl_sum(words, lane);
        const uint32_t total = readlane(incl, kWave - 1);
        if (Wb + total > capw) fits = false;
        if (fits) wv_expand(pk, mk, lut, w, ent, ce, incl - words, incl, total, dst + Wb, lane);
        Wb += total;
        X += xw;
    }
    if (lane == 0) {
        out_len[unit] = (st == ST_OK) ? 8 * Wb : 0;
        status[unit] = (st != ST_OK) ? st : (fits ? ST_OK : ST_SPACE);
    }
    }  // marked units
    }  // unit loop
}

// ---------------------------------------------------------------------------
// DECODE, indexed two-pass decoder (the default)
// ---------------------------------------------------------------------------
// The record chain (tag -> record length -> next tag) is serial within a unit, so
// the decoder splits it from the byte work:
//   pass 1 (decode_index_kernel) walks every unit's chain once, lane per unit, and
//          leaves a u16 record per 16-B piece (first tag offset, words produced);
//   pass 2 (decode_fill_kernel) gives each unit a wave whose lanes start at their
//          own pieces' first tags (no chain to resolve), take their output word
//          offsets from a scan of the records' word counts, expand into LDS and
//          store coalesced.
// Units pass 2 cannot stage (> kFlPieces pieces; decode_long_unit) belong to the
// window-parallel / serial long-unit decoders, which run beside passes 1 and 2 on the
// side stream; the read-message passes (records in the slot, below) also mark units
// whose slot cannot hold the records kStNeedFull for decode_wave_kernel<kWvMarked>.
//
// Piece records live in a library workspace region (rec_region: kRecStride bytes per
// mid-list entry), not in the caller's output slot, so a unit that ends UNEXPECTED_EOF
// or OUT_OF_SPACE leaves its slot untouched (message.zig:90 errors before any output).
// The read-message passes have no workspace: their gated write pass runs only over
// units whose framed length the walk already verified, and keeps the records at the
// front of the slot (rec = nullptr).
constexpr uint32_t kIxDead = 0xFFFFFFFFu;         // walk position of a lane with nothing (more) to walk
constexpr uint32_t kFlPieces = 320;               // pass-2 window: 64 lanes x 5 pieces
constexpr uint64_t kIxSizeMax = 1ull << 31;       // size-only walk: longer units use decode_lane_kernel
// record bytes per unit: 64 B per 8 rounds (+1 store) of at most kFlPieces * 16 B
constexpr uint32_t kRecStride = 64 * ((kFlPieces * 16 / 64 + 8) / 8);
static_assert(kRecStride == 704, "record region stride");

// The units the indexed decoder's fallback owns (the long-unit decoders): an 8-aligned
// output slot and a packed length pass 2 cannot stage (> kFlPieces pieces). Passes 1
// and 2 leave exactly these units alone, so the fallback can run beside them
// (launch_decode).
__device__ __forceinline__ bool decode_long_unit(const uint8_t* in, uint64_t in_off, uint64_t P, uint8_t* out,
                                                 uint64_t out_off, uint64_t cap) {
    (void)cap;
    if (P == 0 || (reinterpret_cast<uintptr_t>(out + out_off) & 7)) return false;
    const uint64_t s = reinterpret_cast<uintptr_t>(in + in_off) & 15;
    return ((s + P + 15) >> 4) > kFlPieces;
}



// Pass 1, decode_index_kernel: lane l of a wave owns unit l and walks its record
// chain once (message.zig:152-191), lockstep by 64-B input block. Every byte is
// fetched from HBM once: round k's loads are quad-coalesced (4 lanes x 16 B = one
// unit's 64-B block, 16 units per instruction), issued one round ahead into
// registers, and written to the lane-major LDS ring: unit u keeps block k at
// ring_u + 16 and block k-1's last 16 B at ring_u (moved there by u's lane at the
// start of round k): 80 B per lane. Round k walks the tags in [64k - 16, 64k + 48), i.e.
// pieces 4k-1 .. 4k+2, whose count bytes (+1, +9) are all resident; a final round
// (k = rounds) walks the last piece.
//
// Per piece p the walk yields a u16 record — the offset of the first tag that
// starts in p (4 bits) | the words its records produce << 4 (0: no tag) — kept at
// index p + 1 of the unit's record array (so a round's four records and a 16-B store
// stay aligned): rec + kRecStride * (list entry) in the workspace, or the front of the
// unit's output slot when rec is null (the read-message gate pass). The walk also
// yields the decoded size and the EOF status.
//
// RD selects the Reader.readPackedMessage passes (reader.zig:84-156; launch_read_message):
//   kRdNone  unpackPacked / estimateUnpackedSize as above;
//   kRdWalk  size-only walk of the kStNeedWalk units that stops at the first record boundary
//            where the decoded words reach out_len[unit] / 8 (the framed length
//            read_header_kernel derived) and writes the bytes it took to consumed[unit]
//            (status kStNeedGate when it reached the framed length exactly);
//   kRdGate  the write pass over in_len = consumed of the kStNeedGate units.
// These take the messages of more than kRdWordsMax framed words; the words decoder takes the
// rest (round 6; round 3's one-walk write pass, kRdOne, was removed with it).
// A unit's status on entry says which pass owns it, so no pass redoes another's work.
constexpr int kRdNone = 0, kRdWalk = 1, kRdGate = 2;

constexpr uint32_t kIxBw = 1;  // waves per block of the index pass (each wave owns 64 units)
// blocks of the index pass for a batch of n units
__host__ __device__ constexpr uint32_t ix_blocks_for(uint32_t n) {
    return (uint32_t)((((uint64_t)n + kWave - 1) / kWave + kIxBw - 1) / kIxBw);
}
template <bool SIZE_ONLY, int RD = kRdNone>
__global__ __launch_bounds__(kWave * kIxBw) void decode_index_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ in_len,
    uint32_t n, uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
    const uint64_t* __restrict__ out_cap, uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
    uint64_t* __restrict__ consumed, const uint32_t* __restrict__ list = nullptr,
    const uint32_t* __restrict__ list_count = nullptr, uint8_t* __restrict__ rec = nullptr) {
    static_assert(RD != kRdWalk || SIZE_ONLY, "the read walk writes no output");
    static_assert(RD != kRdGate || !SIZE_ONLY, "the gated pass is the write pass");
    constexpr bool kStop = RD == kRdWalk;  // the walk stops at the framed length
    constexpr uint32_t kRing = 80;  // [0, 16): block k-1's last piece, [16, 80): block k
    __shared__ __attribute__((aligned(16))) uint8_t ring_blk[kIxBw * kWave * kRing];
    uint8_t* const ring_all = ring_blk + (threadIdx.x >> 6) * (kWave * kRing);  // this wave's
    const uint32_t wv = blockIdx.x * kIxBw + (threadIdx.x >> 6);
    const uint32_t lane = lane_id();
    // with a class list (launch_decode: the mid units), lane l takes list entry 64b + l
    const uint32_t count = list ? *list_count : n;
    if (wv * kWave >= count) return;  // wave-uniform
    const uint32_t slot = wv * kWave + lane;
    const bool valid = slot < count;
    const uint32_t unit = valid ? ((list && count != n) ? list[slot] : slot) : 0u;

    // ---- per-lane unit ---------------------------------------------------------------
    const uint8_t* src = cpk_dummy16;
    uint64_t P64 = 0, cap = 0;
    uint8_t* dstb = nullptr;
    int32_t st = ST_OK;
    bool gated = false;       // RD: another pass owns this unit (or settled it)
    uint64_t lim_w = ~0ull;   // kStop: words of the framed message
    if (valid) {
        if (RD != kRdNone)
            gated = status[unit] != (RD == kRdWalk ? kStNeedWalk : RD == kRdGate ? kStNeedGate : ST_OK);
        src = in + in_off[unit];
        P64 = in_len[unit];
        if (kStop) {
            lim_w = out_len[unit] >> 3;
            // a message of <= 8 Mi + 257 words takes < 2^31 packed bytes (<= 10 B per word),
            // so the walk always stops before this clamp
            if (P64 > kIxSizeMax - 1) P64 = kIxSizeMax - 1;
        }
        if (!SIZE_ONLY) {
            dstb = out + out_off[unit];
            cap = out_cap[unit];
            if (P64 > 0 && (reinterpret_cast<uintptr_t>(dstb) & 7)) st = ST_ARG;  // an empty unit writes nothing
        }
    }
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    bool take = valid && !gated && st == ST_OK && P64 > 0;
    if (take) {
        const uint64_t np = (s + P64 + 15) >> 4;
        const uint64_t nr = (s + P64 + 63) >> 6;  // rounds; records take 16 B per two rounds (+1)
        const bool fits = SIZE_ONLY ? P64 < kIxSizeMax : (np <= kFlPieces && (rec || cap >= 64 * ((nr + 8) / 8)));
        if (!fits) {
            take = false;
            st = kStNeedFull;
        }
    }
    const uint32_t end = take ? s + (uint32_t)P64 : 0u;  // aligned-space end
    const uint32_t npieces = (end + 15) >> 4;
    const uint32_t nr = (end + 63) >> 6;                 // rounds with data for this lane
    uint32_t maxr = nr;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) maxr = max(maxr, (uint32_t)__shfl_xor((int)maxr, d, kWave));
    maxr = __builtin_amdgcn_readfirstlane(maxr);

    // ---- loads: instruction m, lane l moves piece l%4 of unit 16m + l/4's block -------------
    const uint4* qsrc[4];
    uint32_t qlast[4];
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m) {
        const uint32_t r = 16 * m + lane / 4;
        const uint64_t rb = __shfl(reinterpret_cast<uint64_t>(src - s), r, kWave);
        const uint32_t rn = __shfl(npieces, r, kWave);
        qsrc[m] = reinterpret_cast<const uint4*>(rn ? reinterpret_cast<const uint8_t*>(rb) : cpk_dummy16);
        qlast[m] = rn ? rn - 1 : 0u;
    }
    const uint32_t qp = lane & 3;
    u32x4 d0, d1, d2, d3;
    auto load = [&](uint32_t k) {  // asm global loads (ds_gload16): counted by the waits below
        ds_gload16(d0, qsrc[0] + min(4 * k + qp, qlast[0]));
        ds_gload16(d1, qsrc[1] + min(4 * k + qp, qlast[1]));
        ds_gload16(d2, qsrc[2] + min(4 * k + qp, qlast[2]));
        ds_gload16(d3, qsrc[3] + min(4 * k + qp, qlast[3]));
    };
    uint8_t* const wq = ring_all + (lane / 4) * kRing + 16 + 16 * qp;  // unit 16m + l/4: + 16 * kRing * m
    uint8_t* const ring = ring_all + lane * kRing;

    uint32_t pos = take ? s : kIxDead;  // next tag (aligned space)
    uint64_t words = 0;                 // decoded words so far
    uint64_t wrun = 0;                  // kRdWalk: decoded words so far, per record
    uint64_t rec0 = 0;                 // records of the previous (even) round
    u32x4 rq0 = {0, 0, 0, 0}, rq1 = rq0, rq2 = rq0, rq3 = rq0;  // 64 B of records waiting for their store
    uint8_t* const ixp = (!SIZE_ONLY && take) ? (rec ? rec + (uint64_t)kRecStride * slot : dstb) : cpk_sink64;
    const uint32_t nflush = (nr + 8) / 8;  // 64-B record stores of this unit
    if (maxr > 0) load(0);
    for (uint32_t k = 0; k <= maxr; ++k) {
        if (k < maxr) {
            // round k's loads are the oldest in flight; younger: the 4 record stores of round
            // k-1 when it flushed (k-1 = 7 mod 8)
            if (!SIZE_ONLY && (k & 7) == 0 && k > 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
        }
        if (k > 0) {
            wave_lds_sync();  // every lane is done with round k-1's reads
            // the lane's own ring: block k-1's last piece moves to the front (round k
            // reads it for tags in piece 4k-1; the final round k = maxr too)
            *reinterpret_cast<uint4*>(ring) = *reinterpret_cast<const uint4*>(ring + 64);
            wave_lds_sync();  // before the quad writes below overwrite ring + 64
        }
        if (k < maxr) {
            *reinterpret_cast<u32x4*>(wq) = d0;
            *reinterpret_cast<u32x4*>(wq + 16 * kRing) = d1;
            *reinterpret_cast<u32x4*>(wq + 32 * kRing) = d2;
            *reinterpret_cast<u32x4*>(wq + 48 * kRing) = d3;
            if (k + 1 < maxr) load(k + 1);
            wave_lds_sync();
        }
        const uint32_t ob = 64 * k;                 // offset o = pos + 16 - ob in [0, 64)
        const uint32_t lim = min(ob + 48, end);     // tags of pieces 4k-1 .. 4k+2
        uint64_t bits = 0;  // tags that start in pieces 4k-1 .. 4k+2 (bit = offset o)
        uint64_t cnt = 0;   // words of the records of piece 4k-1+i (16-bit field i)
        for (;;) {  // one record per lane per pass; branch-free body, uniform exit
            // a finished or failed lane has pos = kIxDead; a read walk stops at the framed length
            const bool act = pos < lim && (!kStop || wrun < lim_w);
            if (__builtin_amdgcn_ballot_w64(act) == 0) break;
            // ring offset o = pos + 16 - ob: block k-1's last piece at [0, 16), block k at
            // [16, 80); any pos (kIxDead, or past lim) reads inside the lane's ring
            const uint8_t* const a = ring + ((pos + 16u - ob) & 63u);
            uint32_t t = a[0];
            uint32_t b1 = a[1];
            uint32_t c9 = a[9];
            asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));  // one LDS round trip per record
            const bool z = t == 0u, f = t == 0xFFu;
            const uint32_t len = 1u + __popc(t) + (uint32_t)(z | f) + (f ? 8u * c9 : 0u);
            const bool eof = act && pos + len > end;  // message.zig:152-191: record runs past the input
            const bool ok = act && !eof;
            st = eof ? ST_EOF : st;
            const uint32_t o = (pos + 16u - ob) & 63u;
            bits |= (uint64_t)ok << o;
            const uint32_t wd = 1u + (z ? b1 : 0u) + (f ? c9 : 0u);  // <= 256: a piece sums to <= 2048
            cnt += (uint64_t)(ok ? wd : 0u) << (o & 48u);            // field o >> 4
            pos = eof ? kIxDead : (ok ? pos + len : pos);
            if (kStop) wrun += ok ? wd : 0u;
        }
        // every lane stopped (at its framed length, the stream's end or an error)
        const bool stop = kStop && __builtin_amdgcn_ballot_w64(pos < end && wrun < lim_w) == 0;
        if (RD == kRdWalk && stop) break;
        const bool last = k == maxr || stop;
        words += (cnt & 0xFFFFu) + ((cnt >> 16) & 0xFFFFu) + ((cnt >> 32) & 0xFFFFu) + (cnt >> 48);
        if (!SIZE_ONLY) {
            const uint32_t lo = (uint32_t)bits, hi = (uint32_t)(bits >> 32);
            const uint64_t e = (uint64_t)(__builtin_ctz(lo | 0x10000u) & 15u) |
                               ((uint64_t)(__builtin_ctz((lo >> 16) | 0x10000u) & 15u) << 16) |
                               ((uint64_t)(__builtin_ctz(hi | 0x10000u) & 15u) << 32) |
                               ((uint64_t)(__builtin_ctz((hi >> 16) | 0x10000u) & 15u) << 48);
            const uint64_t rec = e | (cnt << 4);  // records 4k .. 4k+3 (pieces 4k-1 .. 4k+2)
            if ((k & 1) || last) {
                // records 8g .. 8g+7 (16 B) go to queue entry g % 4 (a uniform switch: no
                // register indexing); every 8 rounds, and after the last, the queue is stored
                // as 64 contiguous bytes per lane (4 store instructions, which the vmcnt waits
                // above count; lanes without a unit store into cpk_sink64; the slot is 8-B
                // aligned, which gfx950 global stores accept)
                const uint32_t g = k >> 1;
                const uint64_t r0 = (k & 1) ? rec0 : rec, r1 = (k & 1) ? rec : 0ull;
                const u32x4 v = {(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
                switch (g & 3) {
                    case 0: rq0 = v; break;
                    case 1: rq1 = v; break;
                    case 2: rq2 = v; break;
                    default: rq3 = v; break;
                }
                if ((g & 3) == 3 || last) {
                    const uint32_t fb = g >> 2;
                    uint8_t* const q = (take && fb < nflush) ? ixp + 64 * fb : cpk_sink64;
                    // transposed through the ring's first 64 B (round k+1 keeps only its last
                    // 16 B): store m writes units 16m .. 16m+15, 4 lanes x 16 B per unit, so
                    // each instruction writes 16 contiguous 64-B runs, not 64 scattered 16-B ones
                    wave_lds_sync();
                    *reinterpret_cast<u32x4*>(ring) = rq0;
                    *reinterpret_cast<u32x4*>(ring + 16) = rq1;
                    *reinterpret_cast<u32x4*>(ring + 32) = rq2;
                    *reinterpret_cast<u32x4*>(ring + 48) = rq3;
                    wave_lds_sync();
                    const uint64_t qa = reinterpret_cast<uint64_t>(q);
#pragma unroll
                    for (uint32_t m = 0; m < 4; ++m) {
                        const uint32_t u = 16 * m + lane / 4;
                        const uint64_t ua = (uint64_t)(uint32_t)__shfl((int)(uint32_t)qa, (int)u, kWave) |
                                            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(qa >> 32), (int)u, kWave) << 32);
                        const u32x4 v = *reinterpret_cast<const u32x4*>(ring_all + u * kRing + 16 * (lane & 3));
                        uint8_t* const qd = reinterpret_cast<uint8_t*>(ua) + 16 * (lane & 3);
                        asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(qd), "v"(v) : "memory");
                    }
                }
            } else {
                rec0 = rec;
            }
        }
        if (stop) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!valid || gated) return;  // gated: status and out_len of an earlier pass stand
    if (kStop) {
        // reader.zig:91-93 / 146-153: the walk ended at the framed length (OK), past it
        // (InvalidPackedMessage), or the stream ended first (EndOfStream, also for a
        // record cut short: readByte / readNoEof)
        const int32_t rs = (st != ST_OK || wrun < lim_w) ? ST_EOS : (wrun != lim_w ? ST_OVERSHOOT : ST_OK);
        consumed[unit] = rs == ST_OK ? (uint64_t)(pos - s) : 0ull;
        if (rs != ST_OK) {
            out_len[unit] = 0;
            status[unit] = rs;
            return;
        }
        status[unit] = kStNeedGate;  // kRdWalk
        return;
    }
    if (st == kStNeedFull) {
        // the unindexed write pass leaves the unit to the fallback, which owns it from
        // the start (decode_long_unit); the other passes mark it for their successor
        if (SIZE_ONLY || RD != kRdNone) status[unit] = st;
        return;
    }
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    out_len[unit] = 8 * words;
    status[unit] = (!SIZE_ONLY && 8 * words > cap) ? ST_SPACE : ST_OK;
}


constexpr uint32_t kFlWaves = 4;
constexpr uint32_t kFlPk = kFlPieces * 16 + 8;    // staged pieces + room for the 16-B read at the last tag
constexpr uint32_t kFlOut = 512;                  // output words per code pass
constexpr uint32_t kFlMaxL = 5;                   // pieces per lane (kFlPieces / 64)
// Output word codes (u16): a window position q whose byte q is the word's tag and
// bytes q+1 .. q+8 its packed bytes (a mixed record, or an FF record's first word,
// whose tag 0xFF selects all 8 bytes), kFlLit | q for a literal word at q+1 .. q+8
// (an FF run's body), or kFlZero.
// The body of an FF run whose record starts in the pass is left as kFlZero by the code
// walk and filled in afterwards from the FF head before it (fl_bodies).
constexpr uint32_t kFlLit = 0x2000u;
constexpr uint32_t kFlZero = 0xFFFFu;
constexpr uint32_t kFlPos = 0x1FFFu;
static_assert(kFlPk < kFlPos, "codes hold window positions");

// s_waitcnt needs an immediate: wait until at most min(c, 8) vector-memory
// operations are outstanding (a smaller count than the true number of younger
// operations only waits longer).
__device__ __forceinline__ void vmcnt_at_most(uint32_t c) {
    switch (c) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

// Per-unit values the fill pass needs. A wave loads them for 64 of its units at
// once (lane i: the wave's unit k0 + i), so one vector load per array serves 64
// units and each unit reads its values from registers (readlane).
struct FillMeta {
    int32_t st;
    uint32_t P;
    const uint8_t* src;
    uint8_t* dst;
    uint32_t T;  // output words
    const uint16_t* rec;  // piece records
};

// Word of a code (see kFlLit): 16 bytes around its position from the staged
// pieces, then the tag's v_perm selector (literal words: the identity).
__device__ __forceinline__ uint64_t fill_word(const uint8_t* pk, const uint64_t* lut, uint32_t code) {
    if (code == kFlZero) return 0ull;  // a zero word: its lanes issue no LDS reads (p = 0.9: -1%)
    const uint32_t q = code & kFlPos;
    const uint32_t a = q & ~7u, sh = 8u * (q & 7u);
    const uint64_t lo = *reinterpret_cast<const uint64_t*>(pk + a);
    const uint64_t hi = *reinterpret_cast<const uint64_t*>(pk + a + 8);
    const uint32_t t = (code & kFlLit) ? 0xFFu : (uint32_t)(lo >> sh) & 0xFFu;
    const uint64_t pay = ((lo >> sh) >> 8) | (hi << (56u - sh));  // bytes q+1 .. q+8
    return perm64(pay, lut[t]);
}

// FF run bodies of a code pass (message.zig:112-128): the code walk writes only each
// record's first word, so a body's c literal words are still kFlZero, like the words of a
// zero run. Lane l takes codes [8l, 8l + 8): the last written code before each (an
// exclusive max-scan of (index + 1) << 16 | code over the lanes) decides it: after an FF
// head at q (tag byte 0xFF, count c = byte q + 9) the word k words on, k <= c, is the
// literal kFlLit | (q + 1 + 8k); any other kFlZero word is a zero word.
__device__ __forceinline__ void fl_bodies(const uint8_t* pk, uint16_t* code, uint32_t nw, uint32_t lane) {
    uint16_t* const c = code + 8 * lane;  // read from LDS one at a time: few live registers
    uint32_t lh = 0;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        const uint32_t ci = c[i];
        lh = ci != kFlZero ? ((8u * lane + i + 1u) << 16) | ci : lh;
    }
    uint32_t h = fu_prev_lane(wave_incl_max(lh, lane));
    uint32_t body = 0;  // the FF head's count c (0: no body)
    if (h != 0 && !(h & kFlLit)) body = pk[h & kFlPos] == 0xFFu ? pk[(h & kFlPos) + 9] : 0u;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        const uint32_t idx = 8u * lane + i, ci = c[i];
        if (ci != kFlZero) {
            h = ((idx + 1u) << 16) | ci;
            body = !(ci & kFlLit) && pk[ci] == 0xFFu ? pk[ci + 9] : 0u;
        } else if (idx < nw) {
            const uint32_t k = idx + 1u - (h >> 16);
            if (k <= body) c[i] = (uint16_t)(kFlLit | ((h & kFlPos) + 1u + 8u * k));
        }
    }
}

__global__ __launch_bounds__(kFlWaves * kWave) void decode_fill_kernel(const uint8_t* __restrict__ in,
                                                                       const uint64_t* __restrict__ in_off,
                                                                       const uint64_t* __restrict__ in_len,
                                                                       uint32_t n, uint8_t* __restrict__ out,
                                                                       const uint64_t* __restrict__ out_off,
                                                                       const uint64_t* __restrict__ out_len,
                                                                       const uint64_t* __restrict__ out_cap,
                                                                       const int32_t* __restrict__ status,
                                                                       const uint32_t* __restrict__ list = nullptr,
                                                                       const uint32_t* __restrict__ list_count = nullptr,
                                                                       const uint8_t* __restrict__ rec = nullptr) {
    __shared__ __attribute__((aligned(16))) uint8_t pk_all[kFlWaves * kFlPk];
    __shared__ __attribute__((aligned(16))) uint16_t code_all[kFlWaves * (kFlOut + 8)];  // + a dummy slot
    __shared__ uint64_t lut[256];  // tag -> v_perm selector scattering popc(tag) packed bytes
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    lut[threadIdx.x] = expand_selector(threadIdx.x);
    __syncthreads();
    uint8_t* const pk = pk_all + wave * kFlPk;
    uint16_t* const code = code_all + wave * (kFlOut + 8);
    // persistent: the wave takes units u0, u0+G, u0+2G, ... (entries of the class list, if any)
    const uint32_t G = gridDim.x * kFlWaves;
    const uint32_t u0 = blockIdx.x * kFlWaves + wave;
    const uint32_t n_all = n;
    const bool listed = list != nullptr;  // class list: none of its units is the fallback's
    if (list) n = *list_count;
    if (u0 >= n) return;
    if (n == n_all) list = nullptr;  // a list as long as the batch is the identity (batch order)

    uint64_t m_in = 0, m_out = 0, m_rec = 0;  // m_rec: the unit's piece records (decode_index_kernel)
    uint32_t m_P = 0, m_T = 0;
    int32_t m_st = -1;
    auto load_batch = [&](uint32_t k0) {  // meta of the wave's units k0 .. k0+63
        const uint64_t slot = (uint64_t)u0 + (uint64_t)(k0 + lane) * G;
        m_st = -1;
        if (slot < n) {
            const uint32_t uu = list ? list[slot] : (uint32_t)slot;
            m_in = in_off[uu];
            const uint64_t P = in_len[uu];
            m_P = (uint32_t)P;
            m_out = out_off[uu];
            m_rec = reinterpret_cast<uint64_t>(rec ? rec + (uint64_t)kRecStride * slot : out + m_out);
            // the fallback's units (it may be writing their status right now) are skipped
            // without reading what pass 1 left for them (a class list holds none)
            if (listed || !decode_long_unit(in, m_in, P, out, m_out, out_cap[uu])) {
                m_T = (uint32_t)(out_len[uu] >> 3);
                m_st = status[uu];
            }
        }
    };
    auto meta = [&](uint32_t j) {  // the batch's unit j (wave-uniform j)
        FillMeta m;
        m.st = (int32_t)readlane((uint32_t)m_st, j);
        m.P = readlane(m_P, j);
        m.src = in + ((uint64_t)readlane((uint32_t)m_in, j) | ((uint64_t)readlane((uint32_t)(m_in >> 32), j) << 32));
        m.dst = out + ((uint64_t)readlane((uint32_t)m_out, j) | ((uint64_t)readlane((uint32_t)(m_out >> 32), j) << 32));
        m.T = readlane(m_T, j);
        m.rec = reinterpret_cast<const uint16_t*>((uint64_t)readlane((uint32_t)m_rec, j) |
                                                  ((uint64_t)readlane((uint32_t)(m_rec >> 32), j) << 32));
        return m;
    };

    // Registers of the prefetched unit: its pieces (lane l: pieces l + 64m) and the
    // records of the lane's own pieces [lL, lL + L) (decode_index_kernel). Unit k+1 is
    // loaded while unit k is decoded.
    uint4 v0, v1, v2, v3, v4;
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
    auto load_unit = [&](const FillMeta& m) {
        const bool go = m.st == ST_OK && m.P > 0;  // wave-uniform
        if (!go) return;
        const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(m.src) & 15);
        const uint4* const b = reinterpret_cast<const uint4*>(m.src - s);
        const uint32_t np = (s + m.P + 15) >> 4;
        const uint32_t last = np - 1;
        v0 = load_nt(b + min(lane, last));
        if (np > 64) v1 = load_nt(b + min(lane + 64, last));
        if (np > 128) v2 = load_nt(b + min(lane + 128, last));
        if (np > 192) v3 = load_nt(b + min(lane + 192, last));
        if (np > 256) v4 = load_nt(b + min(lane + 256, last));
        const uint32_t L = (np + 63) >> 6;
        const uint16_t* const rc = m.rec;
        const uint32_t q = lane * L + 1;  // record of piece p: index p + 1 (decode_index_kernel)
        r0 = rc[min(q, np)];              // lanes past the last piece read the last record (unused)
        if (L > 1) r1 = rc[min(q + 1, np)];
        if (L > 2) r2 = rc[min(q + 2, np)];
        if (L > 3) r3 = rc[min(q + 3, np)];
        if (L > 4) r4 = rc[min(q + 4, np)];
    };

    load_batch(0);
    FillMeta cur = meta(0);
    load_unit(cur);
    uint32_t younger = 0;  // vector-memory ops issued after cur's loads (its predecessor's stores)
    for (uint32_t k = 0; (uint64_t)u0 + (uint64_t)k * G < n; ++k) {
        const bool go = cur.st == ST_OK && cur.P > 0;
        vmcnt_at_most(younger);  // cur's pieces and records are in registers
        younger = 0;
        uint32_t np = 0, end = 0, pos = 0, words = 0, jend = 0;
        if (go) {
            const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(cur.src) & 15);
            end = s + cur.P;
            np = (end + 15) >> 4;  // <= kFlPieces (decode_index_kernel)
            wave_lds_sync();       // the previous unit's LDS reads are done
            uint4* const pk4 = reinterpret_cast<uint4*>(pk);
            pk4[lane] = v0;
            if (np > 64) pk4[lane + 64] = v1;
            if (np > 128) pk4[lane + 128] = v2;
            if (np > 192) pk4[lane + 192] = v3;
            if (np > 256) pk4[lane + 256] = v4;
            // ---- lane range [q0, q1): first tag and output words, from the piece records ----
            const uint32_t L = (np + 63) >> 6;
            const uint32_t q0 = min(lane * L, np), q1 = min(q0 + L, np);
            const uint32_t nq = q1 - q0;
            jend = min(16 * q1, end);
            pos = jend;
            const uint32_t rr[kFlMaxL] = {r0, r1, r2, r3, r4};
#pragma unroll
            for (int i = kFlMaxL - 1; i >= 0; --i) {
                const uint32_t r = rr[i];
                const bool has = (uint32_t)i < nq && (r >> 4) != 0;
                words += has ? (r >> 4) : 0u;
                pos = has ? 16 * (q0 + i) + (r & 15u) : pos;
            }
        }
        // the next unit's loads go out before any store of this unit
        const uint32_t k1 = k + 1;
        if ((k1 & 63) == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing of cur in flight but its loads (landed)
            load_batch(k1);
        }
        const FillMeta nxt = meta(k1 & 63);  // st = -1 past the batch end
        load_unit(nxt);
        if (go) {
            const uint32_t incl = wave_incl_sum(words, lane);
            const uint32_t wbase = incl - words;
            const bool a16 = !(reinterpret_cast<uintptr_t>(cur.dst) & 15);
            uint64_t* const dst = reinterpret_cast<uint64_t*>(cur.dst);
            const uint32_t T = cur.T;
            for (uint32_t W0 = 0; W0 < T; W0 += kFlOut) {
                // ---- code walk: every lane lists the source of each of its words in [W0, W1)
                const uint32_t W1 = min(T, W0 + kFlOut);
                wave_lds_sync();  // pieces staged; the previous pass's code reads are done
                reinterpret_cast<uint4*>(code)[lane] = make_uint4(kFlZero * 0x10001u, kFlZero * 0x10001u,
                                                                  kFlZero * 0x10001u, kFlZero * 0x10001u);
                wave_lds_sync();
                const bool mine = words > 0 && wbase < W1 && wbase + words > W0;
                uint32_t p = mine ? pos : jend, w = wbase;
                bool runs = false;  // an FF body starts in this pass (fl_bodies)
                for (;;) {  // one record per lane per pass; predicated body, uniform exit
                    const bool act = p < jend && w < W1;
                    if (__builtin_amdgcn_ballot_w64(act) == 0) break;
                    const uint32_t pp = act ? p : 0u;
                    uint32_t t = pk[pp];
                    uint32_t b1 = pk[pp + 1];
                    uint32_t c9 = pk[pp + 9];
                    asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));
                    const bool z = t == 0u, f = t == 0xFFu;
                    // message.zig:101-141: 00 -> zero word(s) (the list starts as kFlZero), FF ->
                    // its first word (tag 0xFF selects the 8 bytes) + c literal words (fl_bodies),
                    // other tags -> scatter of popc(t) bytes
                    code[(act && !z && w >= W0) ? w - W0 : kFlOut] = (uint16_t)pp;
                    const uint32_t c = f ? c9 : 0u;
                    runs |= act && c != 0u;
                    if (act && c && w < W0) {  // a body continued from an earlier pass (rare)
                        for (uint32_t i = W0 - w; i <= c && w + i < W1; ++i)
                            code[w + i - W0] = (uint16_t)(kFlLit | (pp + 1 + 8 * i));
                    }
                    w = act ? w + 1u + (z ? b1 : 0u) + c : w;
                    p = act ? p + 1u + __popc(t) + (uint32_t)(z | f) + 8u * c : p;
                }
                wave_lds_sync();
                if (__builtin_amdgcn_ballot_w64(runs) != 0) {
                    fl_bodies(pk, code, W1 - W0, lane);
                    wave_lds_sync();
                }
                // ---- expand by output word: coalesced stores straight from registers ----------
                const uint32_t nw = W1 - W0;
                if (a16) {
                    for (uint32_t i = 2 * lane; i < nw; i += 2 * kWave) {
                        const uint32_t cc = *reinterpret_cast<const uint32_t*>(code + i);
                        const uint64_t x0 = fill_word(pk, lut, cc & 0xFFFFu);
                        const uint64_t x1 = fill_word(pk, lut, cc >> 16);
                        if (i + 1 < nw) {  // streaming output: non-temporal
                            const u32x4 v = {(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
                            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + W0 + i));
                        }
                        else dst[W0 + i] = x0;
                    }
                    younger += (nw + 2 * kWave - 1) / (2 * kWave);
                } else {
                    for (uint32_t i = lane; i < nw; i += kWave) dst[W0 + i] = fill_word(pk, lut, code[i]);
                    younger += (nw + kWave - 1) / kWave;
                }
            }
        }
        cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// s_waitcnt needs an immediate: wait until at most min(c, 63) vector-memory operations are
// outstanding (fewer than the true number of younger operations only waits longer).
__device__ __forceinline__ void vmcnt_at_most63(uint32_t c) {
#define CPK_VM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
#define CPK_VM8(B) CPK_VM(B) CPK_VM(B + 1) CPK_VM(B + 2) CPK_VM(B + 3) CPK_VM(B + 4) CPK_VM(B + 5) CPK_VM(B + 6) CPK_VM(B + 7)
    switch (c < 63u ? c : 63u) {
        CPK_VM8(0) CPK_VM8(8) CPK_VM8(16) CPK_VM8(24) CPK_VM8(32) CPK_VM8(40) CPK_VM8(48)
        CPK_VM(56) CPK_VM(57) CPK_VM(58) CPK_VM(59) CPK_VM(60) CPK_VM(61) CPK_VM(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
#undef CPK_VM8
#undef CPK_VM
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_incl_max(v, 0), kWave - 1);
}

// ---------------------------------------------------------------------------
// Single-read decoder (round 5): lane per unit, one output word per step
// ---------------------------------------------------------------------------
// unpackPacked (message.zig:88-145) with the size pass's truncation checks (152-191) made on
// the way. A wave owns 64 units. Their packed bytes stream through the index pass's ring
// (quad-coalesced 16-B loads issued a round ahead: every packed byte is fetched from HBM once);
// round k's window holds the unit's bytes [64k - 16, 64k + 64), and its lane emits every output
// word whose source lies in [64k - 16, 64k + 48), ONE word per step:
//   run == 0        a record at pos, tag t: (00) a zero word, then a zero run of b1 more;
//                   (FF) the 8 bytes after the tag, then a literal run of c9 more words;
//                   (other) the popc(t) bytes after the tag scattered by t (message.zig:101-141);
//   run > 0         one more word of the run: zero (rsel 00, no bytes, any round) or literal
//                   (rsel FF, the 8 bytes at pos).
// Steps run in sub-rounds of kLwS, in two phases:
//   A, the chain: per step three byte reads at pos (tag, +1, +9) give the record's length and
//      the next pos; the step only records the word's payload offset in the ring and its
//      selector tag (a literal word: tag FF one byte earlier; a zero word: tag 00), so the
//      dependency pos -> tag -> length -> pos carries a few instructions and one LDS read;
//   B, the words: each recorded word's 8 payload bytes and its v_perm selector, independent
//      of each other, then into the unit's 128-B output line in LDS.
// A line that fills is flushed whole: eight lanes store it as one 128-B line, eight lines per
// store instruction (MI355X: whole lines from eight units write at ~4.3 TB/s, 64-B runs at 8-B
// offsets at ~1.6 TB/s). A sub-round's words past the line's end wait in
// registers until the flush and then start the next line. The unit's first and last lines are
// flushed in part (only its own words; a slot need not be line aligned).
// Errors (message.zig:152-191): a record that runs past the input leaves pos past the end, and
// a literal run cut short leaves run > 0: the unit is UNEXPECTED_EOF, found at its end, so its
// earlier words may already be in its slot (the two-pass decoder writes nothing for a failed
// unit; capnp_packed_set_all_or_nothing routes mid units to it). Words past out_cap are never
// stored; the unit reports OUT_OF_SPACE with the size it needs.
constexpr uint32_t kLwWaves = 2;   // waves per block (a block shares one selector table)
constexpr uint32_t kLwCarry = 12;  // ring bytes kept from the previous round's block
constexpr uint32_t kLwRing = kLwCarry + 64;  // 76 B per lane (an odd dword stride: fewer bank conflicts)
constexpr uint32_t kLwS = 8;       // steps (words) per sub-round
constexpr uint32_t kLwLine = 16;             // words per output line (128 B; 64-B lines measured 2.57 ms vs 1.92)
constexpr uint32_t kLwLB = 8 * kLwLine;      // line bytes
constexpr uint32_t kLwLanes = kLwLB / 16;    // lanes per line in a flush store
// LDS per 2-wave block: rings 9728 + lines 16384 + flush tables 256 + selector table 128 = 26496 B,
// so six blocks (12 waves) fit a CU: the CU admits at most ~159.7 KB of them (census,
// scripts/dev/lds_census.hip: 6 x 26624 B blocks resident, 6 x 27136 B not; 5 x 32768 B neither).
constexpr uint32_t kLwLds = kLwWaves * kWave * (kLwRing + kLwLB + 2) + 128;
static_assert(kLwLds <= 26624, "six blocks per CU");

template <bool RD>
__global__ __launch_bounds__(kLwWaves * kWave) void decode_words_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ in_len,
    uint32_t n, uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
    const uint64_t* __restrict__ out_cap, uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ list_count,
    const uint32_t* __restrict__ list_lo, uint32_t* __restrict__ bail_count, uint64_t* __restrict__ consumed) {
    __shared__ __attribute__((aligned(16))) uint8_t ring_blk[kLwWaves * kWave * kLwRing];
    __shared__ __attribute__((aligned(16))) uint8_t line_blk[kLwWaves * kWave * kLwLB];  // [lane][slot]
    __shared__ uint16_t ftab_blk[kLwWaves * kWave];  // flush table: lane | lo << 6 | hi << 10, by rank
    // The v_perm selector of tag t (message.zig:134-141: bit k set -> output byte k takes the next
    // packed byte) from two reads of a 16-entry table: nibble n -> its 4 selector bytes (bit k set:
    // packed byte popc(n & (2^k - 1)), else 0x0C = a zero byte) | a mask of its set bytes << 32. The
    // high nibble's bytes then add popc(low nibble). At most 16 distinct addresses per read: no bank
    // conflicts (the 256-entry table had 3-4-way conflicts and 2 KB of LDS).
    __shared__ uint64_t nib[16];
    if (threadIdx.x < 16) {
        const uint64_t e = expand_selector(threadIdx.x);
        uint32_t m = 0;
        for (uint32_t k = 0; k < 4; ++k) m |= ((threadIdx.x >> k) & 1u) ? 0xFFu << (8 * k) : 0u;
        nib[threadIdx.x] = (e & 0xFFFFFFFFull) | ((uint64_t)m << 32);
    }
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wave = threadIdx.x >> 6;
    uint8_t* const ring_all = ring_blk + wave * (kWave * kLwRing);
    uint8_t* const lines = line_blk + wave * (kWave * kLwLB);
    uint8_t* const myline = lines + lane * kLwLB;
    uint16_t* const ftab = ftab_blk + wave * kWave;
    const uint32_t wv = blockIdx.x * kLwWaves + wave;
    const uint32_t lo = list_lo ? *list_lo : 0u;  // the list's entries [lo, *list_count)
    const uint32_t count = (list ? *list_count : n) - lo;
    if (wv * kWave >= count) return;  // wave-uniform
    const uint32_t slot = wv * kWave + lane;
    const bool valid = slot < count;
    const uint32_t unit = valid ? ((list && (lo != 0 || count != n)) ? list[lo + slot] : slot) : 0u;

    // ---- per-lane unit ---------------------------------------------------------------
    const uint8_t* src = cpk_dummy16;
    uint64_t P64 = 0, cap = 0;
    uint8_t* dstb = nullptr;
    int32_t st = ST_OK;
    bool gated = false;  // RD: a unit the reader's other passes own (or that its header settled)
    uint64_t fw = 0;     // RD: words of the framed message (read_header_kernel)
    uint32_t past = 0;   // RD: stream bytes past the walked ones (capped; a cut literal run's test)
    if (valid) {
        if (RD) gated = status[unit] != kStWords;
        src = in + in_off[unit];
        P64 = in_len[unit];
        dstb = out + out_off[unit];
        cap = out_cap[unit];
        if (RD) {
            // reader.zig:84-156 decodes records until the framed length is reached; a message
            // takes at most 10 packed bytes per word (an FF record's first word), so the stream
            // past that is never walked (read_header_kernel routes messages of more than
            // kRdWordsMax words to the walk passes)
            fw = out_len[unit] >> 3;
            if (P64 > 10 * fw) {
                past = P64 - 10 * fw > (1u << 20) ? (1u << 20) : (uint32_t)(P64 - 10 * fw);
                P64 = 10 * fw;
            }
        }
        if (P64 > 0 && (reinterpret_cast<uintptr_t>(dstb) & 7)) st = ST_ARG;  // an empty unit writes nothing
        if (P64 >= kIxSizeMax) st = kStNeedFull;  // positions are u32 (the long-unit decoders own these)
    }
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    const bool take = valid && !gated && st == ST_OK && P64 > 0;
    const uint32_t end = take ? s + (uint32_t)P64 : 0u;  // aligned-space end
    const uint32_t npieces = (end + 15) >> 4;
    uint32_t maxr = (end + 63) >> 6;  // rounds with data for this lane
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) maxr = max(maxr, (uint32_t)__shfl_xor((int)maxr, d, kWave));
    maxr = __builtin_amdgcn_readfirstlane(maxr);
    const uint32_t capw = (uint32_t)min(cap >> 3, (uint64_t)0x7FFFFFFFu);
    // The walk stops after lim_w words: the framed length (RD), else the slot's capacity. A unit
    // still owing input at capw is OUT_OF_SPACE (or UNEXPECTED_EOF further on): it is marked for
    // decode_wave_kernel<kWvMarked>, whose window-parallel walk finds its status and size and
    // writes nothing. A lane never steps more than capw words, and long zero runs go out as whole
    // zero lines, so an expansion-heavy unit (00 FF chains: 256 words per 2 bytes) cannot hold its
    // wave (launch_decode routes slots over kWordsCapMax to the two-pass decoder).
    const uint32_t lim_w = RD ? (uint32_t)min(fw, (uint64_t)0x7FFFFFFFu) : capw;
    // output lines: word 0 of the unit sits in slot s0 of the 128-B line at line0
    const uint32_t s0 = take ? (uint32_t)((reinterpret_cast<uintptr_t>(dstb) >> 3) & (kLwLine - 1)) : 0u;
    const uint64_t line0 = reinterpret_cast<uint64_t>(dstb) - 8ull * s0;

    // ---- loads: instruction m, lane l moves piece l%4 of unit 16m + l/4's block ----------
    const uint4* qsrc[4];
    uint32_t qlast[4];
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m) {
        const uint32_t r = 16 * m + lane / 4;
        const uint64_t rb = __shfl(reinterpret_cast<uint64_t>(src - s), r, kWave);
        const uint32_t rn = __shfl(npieces, r, kWave);
        qsrc[m] = reinterpret_cast<const uint4*>(rn ? reinterpret_cast<const uint8_t*>(rb) : cpk_dummy16);
        qlast[m] = rn ? rn - 1 : 0u;
    }
    const uint32_t qp = lane & 3;
    u32x4 d0, d1, d2, d3;
    auto load = [&](uint32_t k) {
        ds_gload16(d0, qsrc[0] + min(4 * k + qp, qlast[0]));
        ds_gload16(d1, qsrc[1] + min(4 * k + qp, qlast[1]));
        ds_gload16(d2, qsrc[2] + min(4 * k + qp, qlast[2]));
        ds_gload16(d3, qsrc[3] + min(4 * k + qp, qlast[3]));
    };
    // a quad lane's 16 B of unit 16m + l/4's block go to ring offset 12 + 16 qp (4-B aligned only:
    // dword writes, as an unaligned ds_write_b128 is correct but ~3.4x slower)
    uint8_t* const wq = ring_all + (lane / 4) * kLwRing + kLwCarry + 16 * qp;
    auto put16 = [&](uint8_t* p, const u32x4& v) {
        uint32_t* const d = reinterpret_cast<uint32_t*>(p);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    };
    uint8_t* const ring = ring_all + lane * kLwRing;

    // ---- flush: every lane with `want` stores words [lo, hi) of its current line (slot
    // range) to the line at address A; eight lanes per line, eight lines per instruction ----
    uint32_t younger = 0;  // store instructions issued after the ring loads in flight
    auto flush = [&](bool want, uint64_t A, uint32_t lo, uint32_t hi) {
        const uint64_t F = __builtin_amdgcn_ballot_w64(want);
        if (F == 0) return;
        const uint32_t cnt = (uint32_t)__popcll(F);
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(F >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)F, 0u));
        wave_lds_sync();  // the previous flush's table reads are done
        if (want) ftab[rk] = (uint16_t)(lane | (lo << 6) | (hi << 10));
        wave_lds_sync();
        const uint32_t Alo = (uint32_t)A, Ahi = (uint32_t)(A >> 32);
        const uint32_t j = lane & (kLwLanes - 1);
        // one pass stores two groups of eight lines; both groups' table, address and line reads
        // go out before either group's stores (the stores carry no memory clobber)
        auto store16 = [&](uint32_t ent, uint64_t a, const u32x4& v, bool in_r) {
            const uint32_t flo = (ent >> 6) & 15u, fhi = ent >> 10;
            uint8_t* const p = reinterpret_cast<uint8_t*>(a) + 16 * j;
            // every line of the group whole (all but a unit's first and last lines): one store
            if (__builtin_amdgcn_ballot_w64(in_r && (flo | (fhi ^ kLwLine)) != 0u) == 0) {
                ++younger;
                if (in_r) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v));
                return;
            }
            const bool a0 = in_r && 2 * j >= flo && 2 * j < fhi, a1 = in_r && 2 * j + 1 >= flo && 2 * j + 1 < fhi;
            const bool both = a0 && a1, first = a0 && !a1, second = a1 && !a0;
            if (__builtin_amdgcn_ballot_w64(both) != 0) {
                ++younger;
                if (both) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v));
            }
            if (__builtin_amdgcn_ballot_w64(first | second) != 0) {
                ++younger;
                uint8_t* const q = second ? p + 8 : p;
                const uint64_t x = second ? ((uint64_t)v.z | ((uint64_t)v.w << 32)) : ((uint64_t)v.x | ((uint64_t)v.y << 32));
                if (first | second) asm volatile("global_store_dwordx2 %0, %1, off nt\n\ts_nop 1" ::"v"(q), "v"(x));
            }
        };
        constexpr uint32_t kGrp = kWave / kLwLanes;  // lines per store instruction
        for (uint32_t g = 0; g < cnt; g += 2 * kGrp) {  // wave-uniform
            const uint32_t ra = g + lane / kLwLanes, rb = ra + kGrp;
            const uint32_t ea = ftab[min(ra, cnt - 1)], eb = ftab[min(rb, cnt - 1)];
            const uint32_t ua = ea & 63u, ub = eb & 63u;
            const uint64_t aa = (uint64_t)(uint32_t)__shfl((int)Alo, (int)ua, kWave) |
                                ((uint64_t)(uint32_t)__shfl((int)Ahi, (int)ua, kWave) << 32);
            const uint64_t ab = (uint64_t)(uint32_t)__shfl((int)Alo, (int)ub, kWave) |
                                ((uint64_t)(uint32_t)__shfl((int)Ahi, (int)ub, kWave) << 32);
            const u32x4 va = *reinterpret_cast<const u32x4*>(lines + ua * kLwLB + 16 * j);
            const u32x4 vb = *reinterpret_cast<const u32x4*>(lines + ub * kLwLB + 16 * j);
            store16(ea, aa, va, ra < cnt);
            if (g + kGrp < cnt) store16(eb, ab, vb, rb < cnt);
        }
    };
    // the slots of line L a flush may store: the unit's own words (from s0 in line 0) below capw
    auto line_hi_cap = [&](uint32_t L, uint32_t hi) {
        const int64_t c = (int64_t)capw + s0 - (int64_t)kLwLine * L;  // slots of line L below word capw
        return (uint32_t)max<int64_t>(0, min<int64_t>(hi, c));
    };

    // Round k's ring holds aligned-space positions [64k - 12, 64k + 64): the 12 carried bytes, then
    // block k at offset 12. A source needs at most its 10 bytes (tag, count/payload), so round k walks
    // the sources below position 64k + 52 (ring offset 64). Positions are kept as ring offsets: the
    // next source's (po) and the unit end's (end_o), both moved back by 64 at every new round.
    constexpr int32_t kFar = 0x3FFFFFFF;                   // a lane with nothing to walk
    int32_t po = take ? (int32_t)(s + kLwCarry) : kFar;    // round 0: ring offset 0 is position -12
    int32_t end_o = take ? (int32_t)(end + kLwCarry) : 0;
    uint32_t run = 0, rsel = 0;  // words left in the current run; its selector tag (00 / FF)
    int32_t apos = po;           // po, or INT_MIN during a zero run (its words need no bytes)
    uint32_t W = 0;              // words emitted
    if (maxr > 0) load(0);
    uint32_t ksh = 0;  // rounds that moved the ring offsets back by 64
    for (uint32_t k = 0; k <= maxr; ++k) {
        // every lane done (input walked, or lim_w words out): the rounds left would only move bytes
        if (__builtin_amdgcn_ballot_w64(take && W < lim_w && (po < end_o || run != 0u)) == 0) break;
        if (k < maxr) {
            vmcnt_at_most63(younger);  // round k's loads are in
            asm volatile("" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
        }
        younger = 0;
        if (k > 0) {
            wave_lds_sync();
            uint32_t* const rd = reinterpret_cast<uint32_t*>(ring);
            const uint32_t c0 = rd[16], c1 = rd[17], c2 = rd[18];  // ring[64, 76) -> ring[0, 12)
            rd[0] = c0;
            rd[1] = c1;
            rd[2] = c2;
            wave_lds_sync();
            po -= 64;
            end_o -= 64;
            ++ksh;
            apos = apos == INT32_MIN ? apos : po;
        }
        if (k < maxr) {
            put16(wq, d0);
            put16(wq + 16 * kLwRing, d1);
            put16(wq + 32 * kLwRing, d2);
            put16(wq + 48 * kLwRing, d3);
            if (k + 1 < maxr) load(k + 1);
            wave_lds_sync();
        }
        const int32_t lim = min(64, end_o);  // sources of this round: ring offsets < lim
        // A lane whose sources below lim are done may go on to ring offsets 64..66 while other
        // lanes finish the round (a source's 10 bytes still lie in the ring; the carry keeps
        // offsets 64.. for the next round), so its next round starts further on
        const int32_t slim = min(67, end_o);
        for (;;) {  // sub-rounds
            // ---- long zero runs: whole zero lines straight to the slot, not a step per word (an
            // expansion-heavy unit, 00 FF: 256 words per 2 bytes, would hold its wave's round) ----
            if (__builtin_amdgcn_ballot_w64(run >= kLwLine && rsel == 0u) != 0) {  // rare: one test per sub-round
                const uint32_t wcap = min(lim_w, capw);  // whole lines below the slot's capacity
                const bool bz = rsel == 0u && run >= kLwLine && ((s0 + W) & (kLwLine - 1)) == 0u &&
                                W + kLwLine <= wcap;
                if (__builtin_amdgcn_ballot_w64(bz) != 0) {
                    const uint32_t nl = bz ? min(run, wcap - W) / kLwLine : 0u;
                    const uint32_t nmax = wave_max_u32(nl);
                    const u32x4 z = {0u, 0u, 0u, 0u};
                    for (uint32_t i = 0; i < nmax; ++i) {  // wave-uniform
                        if (i < nl) {
                            uint8_t* const zl = reinterpret_cast<uint8_t*>(line0 + (uint64_t)kLwLB * ((s0 + W) / kLwLine + i));
#pragma unroll
                            for (uint32_t c = 0; c < kLwLB / 16; ++c)
                                asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(zl + 16 * c), "v"(z));
                        }
                        younger += kLwLB / 16;
                    }
                    W += kLwLine * nl;
                    run -= kLwLine * nl;
                    apos = (run != 0u && rsel == 0u) ? INT32_MIN : po;
                }
            }
            // ---- A: the chain. Step j leaves (payload ring offset | selector tag << 8) in rec[j] ----
            uint32_t rec[kLwS];
#pragma unroll
            for (uint32_t j = 0; j < kLwS; ++j) rec[j] = 0u;  // steps not taken: ring offset 0, tag 00
            uint32_t e = 0;
            // the chain is every lane's critical path: raised wave priority lets it issue ahead of
            // the other waves' phase-B expansion on the SIMD (A/B in profiles/r06_experiments/
            // words_setprio_ab.log: 1-2 % at every density)
            __builtin_amdgcn_s_setprio(1);
            // a decode stops a lane at the first sub-round that ends at or past its capacity (words
            // past out_cap are never stored); a read stops at the framed length exactly
            const uint32_t rem = W < lim_w ? lim_w - W : 0u;
            const int32_t limx = rem != 0u ? slim : INT32_MIN;
#pragma unroll
            for (uint32_t j = 0; j < kLwS; ++j) {
                const bool act = apos < limx && (!RD || j < rem);
                if (__builtin_amdgcn_ballot_w64(act) == 0) break;
                if (act) {
                    // the source's ring offset, kept inside the ring (a zero run's may have left it)
                    const uint32_t o = (uint32_t)min(max(po, 0), 66);
                    const uint8_t* const a = ring + o;
                    uint32_t t = a[0], b1 = a[1], c9 = a[9];
                    asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));  // one LDS round trip per step
                    const bool inrec = run == 0u;
                    const bool tz = t == 0u, tf = t == 0xFFu;
                    const uint32_t len = (uint32_t)__popc(t) + 1u + (uint32_t)(tz | tf);
                    const uint32_t cnt = tz ? b1 : (tf ? c9 : 0u);
                    const uint32_t tsel = inrec ? t : rsel;
                    rec[j] = (o + (uint32_t)inrec) | (tsel << 8);
                    po += (int32_t)(inrec ? len : (rsel & 8u));
                    run = inrec ? cnt : run - 1u;
                    rsel = inrec ? (tf ? 0xFFu : 0u) : rsel;
                    apos = (run != 0u && rsel == 0u) ? INT32_MIN : po;
                    e = j + 1;
                }
            }
            __builtin_amdgcn_s_setprio(0);
            // ---- B: the words (selectors looked up and applied off the chain) ----
            uint64_t w[kLwS];
#pragma unroll
            for (uint32_t j = 0; j < kLwS; ++j) {
                const uint32_t r16 = rec[j];
                const uint32_t o = r16 & 0xFFu, sh = o & 3u;
                const uint32_t* const rw = reinterpret_cast<const uint32_t*>(ring + (o & ~3u));
                const uint32_t D0 = rw[0], D1 = rw[1], D2 = rw[2];
                const uint64_t pay = (uint64_t)__builtin_amdgcn_alignbyte(D1, D0, sh) |
                                     ((uint64_t)__builtin_amdgcn_alignbyte(D2, D1, sh) << 32);
                const uint32_t tg = r16 >> 8;
                const uint64_t elo = nib[tg & 15u], ehi = nib[tg >> 4];
                const uint32_t shi = (uint32_t)ehi + (((uint32_t)__popc(tg & 15u) * 0x01010101u) & (uint32_t)(ehi >> 32));
                w[j] = perm64(pay, (uint64_t)(uint32_t)elo | ((uint64_t)shi << 32));
            }
            // ---- into the unit's line; a line that fills is flushed, the rest follows ----
            const uint32_t sl = (s0 + W) & (kLwLine - 1);  // first slot of this sub-round's words
            const uint32_t f = kLwLine - sl;     // free slots of the current line
#pragma unroll
            for (uint32_t j = 0; j < kLwS; ++j)
                if (j < e && j < f) *reinterpret_cast<uint64_t*>(myline + 8 * ((sl + j) & (kLwLine - 1))) = w[j];
            const bool full = e >= f && e != 0u;
            if (__builtin_amdgcn_ballot_w64(full) != 0) {
                __builtin_amdgcn_s_setprio(1);  // so is the flush the block waits for
                const uint32_t L = (s0 + W) / kLwLine;
                flush(full, line0 + (uint64_t)kLwLB * L, L == 0 ? s0 : 0u, line_hi_cap(L, kLwLine));
                __builtin_amdgcn_s_setprio(0);
                wave_lds_sync();  // the flush's line reads come before the next line's words
#pragma unroll
                for (uint32_t j = 0; j < kLwS; ++j)
                    if (j < e && j >= f) *reinterpret_cast<uint64_t*>(myline + 8 * ((sl + j) & (kLwLine - 1))) = w[j];
            }
            W += e;
            if (__builtin_amdgcn_ballot_w64(apos < lim && W < lim_w) == 0) break;
        }
    }
    // the unit's last line, in part (a full last line went out when it filled)
    {
        const uint32_t L = (s0 + W) / kLwLine, hi = (s0 + W) & (kLwLine - 1);
        const bool part = take && hi != 0u;
        flush(part, line0 + (uint64_t)kLwLB * L, L == 0 ? s0 : 0u, line_hi_cap(L, hi));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!valid || gated) return;
    if (st == kStNeedFull) {  // the long-unit decoders' (launch_decode never lists these here)
        status[unit] = st;
        return;
    }
    if (RD) {
        // reader.zig:91-93 / 146-153: the walk stopped at the first record boundary with the framed
        // length reached (OK, consumed = the bytes it took), inside a run that passes it
        // (InvalidPackedMessage, unless the run's literal bytes are cut: readNoEof's EndOfStream),
        // or the stream ended first / cut a record (EndOfStream)
        const int32_t rend = po + (int32_t)((rsel & 8u) * run);  // the current record's end
        int32_t rs = st;
        if (rs == ST_OK && take)
            rs = (W < lim_w || po > end_o) ? ST_EOS
                                           : (run != 0u ? (rend > end_o + (int32_t)past ? ST_EOS : ST_OVERSHOOT) : ST_OK);
        if (rs != ST_OK) {
            out_len[unit] = 0;
            consumed[unit] = 0;
            status[unit] = rs;
            return;
        }
        // aligned-space position: po + 64 per round that moved it back, less the carry's offset
        consumed[unit] = take ? (uint64_t)((int64_t)po + 64ll * ksh - kLwCarry - s) : 0ull;
        out_len[unit] = 8ull * W;
        status[unit] = 8ull * W > cap ? ST_SPACE : ST_OK;
        return;
    }
    // message.zig:152-191: the walk ends exactly at the input's end with no literal word owed;
    // a unit stopped at capw with input left needs its status and size from the fallback walk
    if (take && (po != end_o || run != 0u)) {
        if (W >= lim_w && po <= end_o) {
            status[unit] = kStNeedFull;  // decode_wave_kernel<kWvMarked>: status and size, no output
            atomicAdd(bail_count, 1u);
            return;
        }
        st = ST_EOF;
    }
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    out_len[unit] = 8ull * W;
    status[unit] = 8ull * W > cap ? ST_SPACE : ST_OK;
}

// The earlier single-read mid-unit decoders (fused, round 3; streaming, round 4) measured slower
// than the two-pass decoder and were removed in round 5; their source is at 869fccf
// (csrc/dev_decoders.inc).

// ---- size classes ------------------------------------------------
// A batch's units are split by size before the coding kernels run, so each kernel gets
// units of the shape it is built for:
//   small: lane per unit (encode_stream_kernel / decode_small_kernel): units so short that
//          a wave per unit would leave most of its 64 lanes idle (config C5: median 15 words);
//   mid:   a wave per unit (encode_kernel) / the words decoder (decode_words_kernel, a lane
//          per unit) or the indexed decoder (decode_index_kernel, 64 units per wave, then
//          decode_fill_kernel, a wave per unit);
//   long, huge: a wave per unit walking it tile by tile / window by window
//          (encode_tiled_kernel / decode_wave_kernel<kWvLong>), on the side stream.
// Workspace q (queue_bytes(n)): q[0] long, q[2] huge, q[3] small and q[4] mid counts, q[5]
// serial units, q[8..9] tiles / windows listed, q[10] serial take cursor, q[11 + b] mid units before bin b; the long list at q[kQHead ..] upwards and the huge list from
// q[kQHead + n - 1] downwards, the small list at q[kQHead + n ..], the mid list at
// q[kQHead + 2n ..], kClassK counts per class block, the serial list (serial_off), then the
// tile table (encode) or the window table (decode). Count, scan, scatter: each list keeps
// batch order, and no atomic is contended.
// decode mid units are binned by packed length (CL_MID + 0..7: <= 768, 1024, 1280, 1536, 2048,
// 2560, 3072, more bytes), so the lanes of an index-pass or words-decoder wave walk units of
// similar length in lockstep; the mid list is the bins in order (batch order within a bin), and
// q[20] is the two-pass decoder's share of it (class_scan_kernel).
enum : uint32_t { CL_LONG = 0, CL_HUGE = 1, CL_SMALL = 2, CL_MID = 3, CL_MID_BINS = 8 };
constexpr uint32_t kEsBinsQ = 4;  // encode's small-unit bins (mid-list bins 4 .. 7, kEsBins)
constexpr uint64_t kSmEncWords = 64;  // encode: units of at most 64 words are small
constexpr uint64_t kSmDecP = 512;     // decode: small = at most 512 packed bytes ...
constexpr uint64_t kSmDecCap = 8192;  // ... into a slot of at most 8 KiB
constexpr uint64_t kMidSplitP = 1280; // decode: mid units of at most this many packed bytes (bins 0 .. 2)
constexpr uint64_t kWordsCapMax = 8192;  // decode: the words decoder takes slots of at most 8 KiB

__device__ __forceinline__ uint32_t* q_blocks(uint32_t* q, uint32_t n) { return q + kQHead + 3ull * n; }

// KIND 1: decode (small lane kernel + words / indexed mid decoders), 2: decoded size (no output:
// long by packed length alone), 4: encode with the streaming small-unit encoder (mid units bin
// 0, small units bins 4 .. 7)
template <int KIND>
__device__ __forceinline__ uint32_t unit_class(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                               uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                                               uint32_t u) {
    const uint64_t off = in_off[u], len = in_len[u];
    if (KIND == 2) {
        const uint64_t s = reinterpret_cast<uintptr_t>(in + off) & 15;
        if (len > 0 && ((s + len + 15) >> 4) > kFlPieces) return len > kQHuge ? CL_HUGE : CL_LONG;
        return CL_MID;
    }
    if (KIND == 4) {
        if (encode_tiled_unit(in, off, len)) return len > kQHuge ? CL_HUGE : CL_LONG;
        const bool valid = !(reinterpret_cast<uintptr_t>(in + off) & 7) && !(len & 7);
        const bool small = !valid || (len >> 3) <= kSmEncWords;
        const uint64_t w = len >> 3;
        return !small ? CL_MID : CL_MID + 4 + (valid && w > 8) + (valid && w > 16) + (valid && w > 32);
    }
    const uint64_t cap = out_cap[u];
    if (len <= kSmDecP && cap <= kSmDecCap) return CL_SMALL;
    if (decode_long_unit(in, off, len, out, out_off[u], cap)) return len > kQHuge ? CL_HUGE : CL_LONG;
    // a slot over kWordsCapMax: the two-pass decoder's bins (its fill expands a unit 64 words per
    // step; the words decoder steps a word at a time, up to capw of them)
    if (cap > kWordsCapMax) return CL_MID + (len > 768) + (len > 1024);
    return CL_MID + (len > 768) + (len > 1024) + (len > kMidSplitP) + (len > 1536) + (len > 2048) + (len > 2560) +
           (len > 3072);
}

// Pass 1: units per class in each block of kClassBlock units; long units get the
// kStPending sentinel until their worker writes their outcome (a unit the worker never
// reached shows DEVICE_ERROR, not a stale status).
template <int KIND>
__global__ __launch_bounds__(kClassBlock) void class_count_kernel(const uint8_t* __restrict__ in,
                                                                  const uint64_t* __restrict__ in_off,
                                                                  const uint64_t* __restrict__ in_len, uint32_t n,
                                                                  uint8_t* __restrict__ out,
                                                                  const uint64_t* __restrict__ out_off,
                                                                  const uint64_t* __restrict__ out_cap, uint32_t* q,
                                                                  int32_t* __restrict__ status) {
    __shared__ uint32_t cnt[kClassK];
    if (threadIdx.x < kClassK) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t u = blockIdx.x * kClassBlock + threadIdx.x;
    const uint32_t c = u < n ? unit_class<KIND>(in, in_off, in_len, out, out_off, out_cap, u) : kClassK;
    if (c <= CL_HUGE) status[u] = kStPending;
#pragma unroll
    for (uint32_t k = 0; k < kClassK; ++k) {
        const uint64_t m = __ballot(c == k);
        if (m && lane_id() == 0) atomicAdd(&cnt[k], (uint32_t)__popcll(m));  // LDS
    }
    __syncthreads();
    if (threadIdx.x < kClassK) q_blocks(q, n)[blockIdx.x * kClassK + threadIdx.x] = cnt[threadIdx.x];
}

// Pass 2 (one block): exclusive scan of the block counts per class, and the totals.
__global__ __launch_bounds__(1024) void class_scan_kernel(uint32_t* q, uint32_t n, uint32_t nb, uint32_t words_min) {
    __shared__ uint32_t wsum[16][kClassK];
    __shared__ uint32_t carry[kClassK];
    uint32_t* const bl = q_blocks(q, n);
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    if (threadIdx.x < kClassK) carry[threadIdx.x] = 0;
    // the workspace head: every counter and cursor zero before the entries below are set (was a
    // memset on the caller's stream, one more launch per batch; nothing reads the head between
    // the workspace's hand-out and this kernel)
    if (threadIdx.x < kQHead) q[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t b = b0 + threadIdx.x;
        uint32_t v[kClassK], incl[kClassK];
#pragma unroll
        for (uint32_t k = 0; k < kClassK; ++k) {
            v[k] = b < nb ? bl[b * kClassK + k] : 0u;
            incl[k] = wave_incl_sum(v[k], lane);
            if (lane == 63) wsum[w][k] = incl[k];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < kClassK; ++k) {
            uint32_t pre = carry[k];
            for (uint32_t j = 0; j < w; ++j) pre += wsum[j][k];
            if (b < nb) bl[b * kClassK + k] = pre + incl[k] - v[k];
        }
        __syncthreads();
        if (threadIdx.x < kClassK) {
            uint32_t t = 0;
            for (uint32_t j = 0; j < 16; ++j) t += wsum[j][threadIdx.x];
            carry[threadIdx.x] += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        q[0] = carry[CL_LONG];
        q[2] = carry[CL_HUGE];
        q[3] = carry[CL_SMALL];
        uint32_t mid = 0;  // q[11 + b]: mid units in the bins before bin b
        for (uint32_t b = 0; b < CL_MID_BINS; ++b) {
            q[11 + b] = mid;
            mid += carry[CL_MID + b];
        }
        q[4] = mid;
        // decode: the mid list's share for the two-pass decoder, [0, q[20]); the words decoder
        // takes [q[20], mid). words_min 0: all to the words decoder; else the units over
        // kMidSplitP packed bytes (bins 3 .. 7) when there are at least words_min of them
        // (the words decoder is a throughput design, and a wave's walk of
        // ~600 steps is long: under a resident grid of units, or at p ~ 0.9, two-pass wins)
        const uint32_t over = mid - q[11 + 3];
        q[20] = words_min == 0 ? 0u : (over >= words_min ? q[11 + 3] : mid);
        q[21] = 0;  // decode_words_kernel's count of units stopped at their slot's capacity
    }
}

// Pass 3: every unit to its place in its class list (batch order within a class).
// fused (a batch of at most kClassBlock class blocks): class_scan_kernel is not launched; every
// block sums the per-block counts itself (a thread per class block: the counts of the blocks
// before it and the totals), and block 0 writes the workspace head the scan would have. One
// launch and its dependency gap fewer per batch call for ~48 KB of L2 reads per block.
template <int KIND>
__global__ __launch_bounds__(kClassBlock) void class_scatter_kernel(const uint8_t* __restrict__ in,
                                                                    const uint64_t* __restrict__ in_off,
                                                                    const uint64_t* __restrict__ in_len, uint32_t n,
                                                                    uint8_t* __restrict__ out,
                                                                    const uint64_t* __restrict__ out_off,
                                                                    const uint64_t* __restrict__ out_cap, uint32_t* q,
                                                                    uint32_t fused, uint32_t words_min) {
    __shared__ uint32_t wcnt[16][kClassK];
    __shared__ uint32_t wtot[16][kClassK];
    __shared__ uint32_t pre_s[kClassK], own_s[kClassK], tot_s[kClassK], midb_s[CL_MID_BINS + 1];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t u = blockIdx.x * kClassBlock + threadIdx.x;
    const uint32_t nb = gridDim.x;
    // fused: thread t holds class block t's counts, loaded beside the unit's own metadata
    uint32_t v[kClassK];
    if (fused) {  // block-uniform; nb <= kClassBlock (launch_classes)
        const uint32_t* const bl = q_blocks(q, n);
#pragma unroll
        for (uint32_t k = 0; k < kClassK; ++k) v[k] = threadIdx.x < nb ? bl[threadIdx.x * kClassK + k] : 0u;
    }
    const uint32_t c = u < n ? unit_class<KIND>(in, in_off, in_len, out, out_off, out_cap, u) : kClassK;
    if (fused) {  // one block-wide inclusive scan per class: this block's exclusive prefix, the totals
#pragma unroll
        for (uint32_t k = 0; k < kClassK; ++k) {
            const uint32_t a = wave_incl_sum(v[k], lane);
            if (lane == 63) wtot[w][k] = a;
            if (threadIdx.x == blockIdx.x) {
                own_s[k] = v[k];
                pre_s[k] = a - v[k];  // within its wave; the waves before it are added below
            }
        }
    }
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t k = 0; k < kClassK; ++k) {
        const uint64_t m = __ballot(c == k);
        if (lane == 0) wcnt[w][k] = (uint32_t)__popcll(m);
        if (c == k) rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    __syncthreads();
    if (fused) {
        if (threadIdx.x < kClassK) {
            const uint32_t wb = blockIdx.x >> 6;  // the wave holding this block's counts
            uint32_t a = 0, b = 0;
            for (uint32_t j = 0; j < 16; ++j) {
                a += wtot[j][threadIdx.x];
                b += j < wb ? wtot[j][threadIdx.x] : 0u;
            }
            tot_s[threadIdx.x] = a;
            pre_s[threadIdx.x] += b;
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // q[11 + b]: mid units in the bins before bin b (class_scan_kernel)
            uint32_t mid = 0;
            for (uint32_t b = 0; b < CL_MID_BINS; ++b) {
                midb_s[b] = mid;
                mid += tot_s[CL_MID + b];
            }
            midb_s[CL_MID_BINS] = mid;
        }
        __syncthreads();
        if (blockIdx.x == 0 && threadIdx.x < kQHead) {  // the head, as class_scan_kernel writes it
            const uint32_t t = threadIdx.x, mid = midb_s[CL_MID_BINS];
            uint32_t v = 0;
            if (t == 0) v = tot_s[CL_LONG];
            else if (t == 2) v = tot_s[CL_HUGE];
            else if (t == 3) v = tot_s[CL_SMALL];
            else if (t == 4) v = mid;
            else if (t >= 11 && t < 11 + CL_MID_BINS) v = midb_s[t - 11];
            else if (t == 20) v = words_min == 0 ? 0u : (mid - midb_s[3] >= words_min ? midb_s[3] : mid);
            q[t] = v;
        }
    }
    if (c >= kClassK) return;
    const uint32_t* const P = q_blocks(q, n);  // exclusive prefixes over blocks, per class (scanned)
    const uint32_t pc = fused ? pre_s[c] : P[blockIdx.x * kClassK + c];
    uint32_t idx = pc + rank;
    for (uint32_t j = 0; j < w; ++j) idx += wcnt[j][c];
    if (KIND == 4 && c >= CL_MID + CL_MID_BINS - kEsBinsQ) {
        // encode's small units ordered by (class block, length bin) instead of (bin, batch order):
        // a unit's neighbours in memory (other bins) are then coded by waves of the same block,
        // at about the same time, so the lines they share are read once
        uint32_t before = 0;  // small units of earlier blocks, and of lower bins in this block
        for (uint32_t cc = CL_MID + CL_MID_BINS - kEsBinsQ; cc < CL_MID + CL_MID_BINS; ++cc) {
            const uint32_t b = cc - CL_MID;
            uint32_t pb, pn;
            if (fused) {
                pb = pre_s[cc];
                pn = pb + own_s[cc];
            } else {
                const uint32_t tot = (b + 1 < CL_MID_BINS ? q[12 + b] : q[4]) - q[11 + b];
                pb = P[blockIdx.x * kClassK + cc];
                pn = blockIdx.x + 1 < nb ? P[(blockIdx.x + 1) * kClassK + cc] : tot;
            }
            before += pb + (cc < c ? pn - pb : 0u);
        }
        idx = before + (idx - pc);
        const uint32_t base = fused ? midb_s[CL_MID_BINS - kEsBinsQ] : q[11 + CL_MID_BINS - kEsBinsQ];
        q[kQHead + 2ull * n + base + idx] = u;
        return;
    }
    if (c == CL_LONG) q[kQHead + idx] = u;
    else if (c == CL_HUGE) q[kQHead + n - 1 - idx] = u;
    else if (c == CL_SMALL) q[kQHead + 1ull * n + idx] = u;
    else q[kQHead + 2ull * n + (fused ? midb_s[c - CL_MID] : q[11 + (c - CL_MID)]) + idx] = u;
}

// ---- long units, tile-parallel encode ---------------------------------
// A long unit's tiles (512 words) are encoded by different waves, each like a mid unit
// (encode_tile), instead of one wave walking the unit tile by tile:
//   long_tiles_kernel  lists every tile of every long unit in a tile table (a unit's
//                      tiles adjacent; a unit that does not fit the table goes to the
//                      serial list, encode_tiled_kernel's);
//   tile_encode_kernel<kTilesSize>   per tile: the runs open at its start (the last
//                      zero-run / literal-run break before it, read backwards from the
//                      input: the carries encode_tiled_kernel passes from tile to tile),
//                      the first breaks after its end (lookahead), its packed size;
//   tile_encode_kernel<kTilesWrite>  per tile: its output offset = the unit's earlier
//                      tiles' sizes (one wave reduction), the tile coded again and
//                      written there; the unit's last tile writes out_len and status.
// The table lives in the class workspace after the class lists: tile sizes (u64), units,
// first tile of the unit; capacity n + kTileExtra tiles.
constexpr uint64_t kTileExtra = 65536;
constexpr uint32_t kTileSkip = 0xFFFFFFFFu;  // a table entry of a unit that went to the serial list
struct TileTab {
    uint64_t* size;
    uint32_t* unit;
    uint32_t* first;
    uint32_t* serial;
    uint64_t cap;
};
__host__ __device__ inline uint64_t tile_tab_off(uint64_t n) {  // u32 index of the tile table (8-B aligned)
    return (serial_off(n) + n + 1) & ~1ull;
}
__device__ __forceinline__ TileTab tile_tab(uint32_t* q, uint32_t n) {
    TileTab t;
    t.cap = (uint64_t)n + kTileExtra;
    t.serial = q + serial_off(n);
    t.size = reinterpret_cast<uint64_t*>(q + tile_tab_off(n));
    t.unit = q + tile_tab_off(n) + 2 * t.cap;
    t.first = t.unit + t.cap;
    return t;
}
// q[5]: serial units; q[8..9]: tiles reserved (u64); q[10]: serial take cursor
__device__ __forceinline__ unsigned long long* q_tiles(uint32_t* q) { return reinterpret_cast<unsigned long long*>(q + 8); }

// Consecutive ranges of a shared counter for a wave's lanes (k each, 0: none), in lane order,
// with ONE atomic per wave: ~10K long units each adding to the one counter serialised at its L2
// channel while the small-unit kernel loaded the memory system (config C5: 0.21 ms).
__device__ __forceinline__ uint64_t wave_reserve(unsigned long long* ctr, uint64_t k) {
    const uint32_t lane = lane_id();
    uint64_t incl = k;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint64_t o = __shfl_up(incl, d, kWave);
        if (lane >= (uint32_t)d) incl += o;
    }
    const uint64_t total = __shfl(incl, kWave - 1, kWave);
    uint64_t b = 0;
    if (lane == 0 && total != 0) b = atomicAdd(ctr, (unsigned long long)total);
    b = __shfl(b, 0, kWave);
    return b + incl - k;
}

__global__ __launch_bounds__(256) void long_tiles_kernel(const uint64_t* __restrict__ in_len, uint32_t n, uint32_t* q) {
    const uint32_t nh = q[2], nl = q[0];
    const TileTab t = tile_tab(q, n);
    // as long_windows_kernel: wave-uniform trips, one reservation per wave
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~(kWave - 1)); i0 < nl + nh; i0 += gridDim.x * 256) {
    const uint32_t i = i0 + lane_id();
    const bool v = i < nl + nh;
    const uint32_t unit = !v ? 0u : (i < nh ? q[kQHead + n - 1 - i] : q[kQHead + (i - nh)]);
    const uint64_t k = v ? ((in_len[unit] >> 3) + kEncMaxWords - 1) / kEncMaxWords : 0ull;  // >= 2 tiles
    const uint64_t r = wave_reserve(q_tiles(q), (v && k <= t.cap) ? k : 0ull);
    if (!v) continue;
    const uint64_t base = k <= t.cap ? r : t.cap;
    if (base + k <= t.cap) {
        for (uint64_t j = 0; j < k; ++j) {
            t.unit[base + j] = unit;
            t.first[base + j] = (uint32_t)base;
        }
    } else {
        for (uint64_t j = base; j < t.cap; ++j) t.unit[j] = kTileSkip;  // reserved past the end: unused
        t.serial[atomicAdd(q + 5, 1u)] = unit;
    }
    }
}

// Last zero-run break (a word that is not zero) and last literal-run break (a word with a
// zero byte) before word tb, as run starts (break + 1; 0: the run starts the unit);
// wave-uniform results. Reads 256 words back at a time (one pass for most data).
__device__ __forceinline__ void encode_lookback(const uint8_t* src, uint32_t tb, uint32_t lane, uint32_t& cz,
                                                uint32_t& cf) {
    uint32_t lz = 0, lf = 0;
    bool fz = false, ff = false;
    uint32_t end = tb;
    while (end > 0 && !(fz && ff)) {  // wave-uniform
        const uint32_t w0 = end > 256 ? end - 256 : 0;
        uint32_t bz = 0, bf = 0;  // last break + 1 among this lane's words
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t i = w0 + 4 * lane + k;
            if (i < end) {
                const uint32_t tg = nonzero_tag(*reinterpret_cast<const uint64_t*>(src + 8ull * i));
                if (tg != 0) bz = i + 1;
                if (tg != 0xFF) bf = i + 1;
            }
        }
        bz = readlane(wave_incl_max(bz, lane), kWave - 1);
        bf = readlane(wave_incl_max(bf, lane), kWave - 1);
        if (!fz && bz) { lz = bz; fz = true; }
        if (!ff && bf) { lf = bf; ff = true; }
        end = w0;
    }
    cz = lz;
    cf = lf;
}

constexpr int kTilesSize = 0, kTilesWrite = 1;
template <int PASS, bool WRITE>
__global__ __launch_bounds__(kBlock) void tile_encode_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ in_off,
                                                             const uint64_t* __restrict__ in_len, uint32_t n,
                                                             uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off,
                                                             const uint64_t* __restrict__ out_cap,
                                                             uint64_t* __restrict__ out_len,
                                                             int32_t* __restrict__ status, uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kEncLds];
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const TileTab t = tile_tab(q, n);
    const uint64_t T = min((uint64_t)*q_tiles(q), t.cap);
    if ((uint64_t)blockIdx.x * kWavesPerBlock >= T) return;  // block-uniform
    constexpr bool CODE = PASS == kTilesSize || WRITE;  // the pass codes tiles (else: totals only)
    if (CODE && PASS == kTilesWrite) {
        lut[threadIdx.x] = compact_selector(threadIdx.x);
        __syncthreads();
    }
    uint8_t* const lds = smem + wave * kEncLds;
    const uint64_t G = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t g = (uint64_t)blockIdx.x * kWavesPerBlock + wave; g < T; g += G) {
        uint32_t lane_g = lane;
        asm volatile("" : "+v"(lane_g));  // lane-derived addresses: recomputed, not held across the loop
        const uint32_t unit = __builtin_amdgcn_readfirstlane(t.unit[g]);
        if (unit == kTileSkip) continue;
        const uint64_t g0 = __builtin_amdgcn_readfirstlane(t.first[g]);
        const uint32_t j = (uint32_t)(g - g0);
        const uint8_t* const src = in + in_off[unit];
        const uint32_t words = (uint32_t)(in_len[unit] >> 3);
        const uint32_t tb = j * kEncMaxWords;
        const uint32_t tw = min(kEncMaxWords, words - tb);
        const uint32_t te = tb + tw;
        const bool last = te == words;
        uint64_t off = 0;  // the tile's output offset: the unit's earlier tiles' sizes
        if (PASS == kTilesWrite) {
            uint64_t acc = 0;
            for (uint32_t b = 0; b < j; b += kWave) {
                const uint32_t i = b + lane_g;
                const uint64_t v = i < j ? t.size[g0 + i] : 0ull;
                acc += v;
            }
            off = wave_sum64(acc);
        }
        uint64_t ob = 0, cap = 0;
        if (WRITE) {
            ob = out_off[unit];
            cap = out_cap[unit];
        }
        if (!CODE) {  // encoded-size pass: the last tile reports the unit's total
            if (last && lane_g == 0) {
                out_len[unit] = off + t.size[g];
                status[unit] = ST_OK;
            }
            continue;
        }
        uint4 v[5];
        encode_load(v, src + 8ull * tb, tw, lane_g);
        uint32_t cz = 0, cf = 0;
        if (tb > 0) encode_lookback(src, tb, lane_g, cz, cf);
        uint32_t nbz = words, nbf = words;
        if (!last) {
            const uint32_t la = min(256u, words - te);
            uint32_t bz, bf;
            encode_lookahead(src + 8ull * te, la, lane_g, bz, bf);
            nbz = bz < la ? te + bz : (la == 256u ? te + 256u : words);
            nbf = bf < la ? te + bf : (la == 256u ? te + 256u : words);
        }
        wave_lds_sync();  // the previous tile's write-back read the slice
        encode_put(lds, v, (uint32_t)(reinterpret_cast<uintptr_t>(src + 8ull * tb) & 15), tw, lane_g);
        wave_lds_sync();
        if (PASS == kTilesSize) {
            const uint32_t P = encode_tile<false, false>(lds, lut, lane_g, tw, tb, cz, cf, nbz, nbf, nullptr, 0);
            if (lane_g == 0) t.size[g] = P;
        } else {
            const uint64_t room = off <= cap ? cap - off : 0;
            const uint32_t P = encode_tile<true, false>(lds, lut, lane_g, tw, tb, cz, cf, nbz, nbf, out + ob + off, room);
            if (last && lane_g == 0) {
                out_len[unit] = off + P;
                status[unit] = off + P > cap ? ST_SPACE : ST_OK;
            }
        }
    }
}

// ---- long units, window-parallel decode ------------------------------
// A long unit's packed bytes are cut into windows of kWvWin bytes at fixed positions
// X_j = j * kWvWin, and every window is a wave's work, instead of one wave walking the
// unit window after window. Where the record chain enters window j is only known once
// window j-1 is resolved, so:
//   long_windows_kernel   lists every window of every long unit in a window table (a
//                         unit's windows adjacent; units that do not fit go to the serial
//                         list, decode_wave_kernel<kWvLong>'s);
//   window_spec_kernel    per window: the chain as if a record started at X_j (walk A/B
//                         and the verification rounds of wv_resolve), its exit and word
//                         count; then, for every possible entry d < kWinD, a walk from d
//                         until it meets a verified record start of lanes 0/1 (chains
//                         couple within a few records): from there its records are the
//                         verified chain's, so the words from entry d are the window's
//                         count plus delta[d];
//   window_resolve_kernel per unit (a wave, serial over its windows but table lookups
//                         only): entry d_0 = 0, d_{j+1} = X_j + exit_j - X_{j+1}, words_j =
//                         total_j + delta_j[d_j]; an entry the spec pass could not resolve
//                         (an FF record landing >= kWinD bytes in, or no coupling within
//                         lanes 0/1) is resolved by staging that window again. It writes
//                         each window's entry and output offset, and the unit's out_len and
//                         status BEFORE any output exists: a truncated or oversized unit
//                         writes nothing (message.zig:90 errors before producing output);
//   window_fill_kernel    per window of an OK unit: the chain from its exact entry, the
//                         code list and the expansion (wv_expand) at its output offset.
// The table shares the class workspace's tile-table region (encode's); capacity
// n / 8 + kWinExtra windows (4.6 KB each).
constexpr uint64_t kWinExtra = 32768;
constexpr uint32_t kWinNone = 0xFFFFFFFFu;  // window entry: nothing to expand
constexpr int16_t kDeltaEof = -32768;       // delta: the chain from this entry runs past the unit's end
constexpr uint32_t kWinD = 64;              // entries the spec pass resolves (window bytes 0 .. 63)
constexpr uint32_t kWinBatch = 32;          // windows whose tables a resolve wave holds at once
struct WinEnt {
    uint32_t unit, first;  // the unit (kTileSkip: none); table index of its first window
    uint32_t exit, total;  // spec pass: exit (window-relative, kEOFX) and words from entry 0
    uint64_t valid;        // spec pass: bit d = delta[d] holds the words from entry d
    uint32_t ent, pad;     // resolve pass: the verified entry (window-relative) or kWinNone
    uint64_t wb;           // resolve pass: output words before the window
    uint64_t pad2;
    int16_t delta[kWinD];  // spec pass: words from entry d - total (kDeltaEof: truncated)
};
static_assert(sizeof(WinEnt) == 176, "window table entry");
__host__ __device__ inline uint64_t win_tab_off(uint64_t n) { return (tile_tab_off(n) + 3) & ~3ull; }  // 16-B aligned
__host__ __device__ inline uint64_t win_cap(uint64_t n) { return n / 8 + kWinExtra; }
__device__ __forceinline__ WinEnt* win_tab(uint32_t* q, uint32_t n) {
    return reinterpret_cast<WinEnt*>(q + win_tab_off(n));
}

__global__ __launch_bounds__(256) void long_windows_kernel(const uint64_t* __restrict__ in_len, uint32_t n,
                                                           uint32_t* q) {
    const uint32_t nh = q[2], nl = q[0];
    WinEnt* const e = win_tab(q, n);
    const uint64_t cap = win_cap(n);
    // a small grid (list_blocks) striding over the long list, wave-uniform trips; the windows
    // are reserved with one atomic per wave (wave_reserve)
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~(kWave - 1)); i0 < nl + nh; i0 += gridDim.x * 256) {
    const uint32_t i = i0 + lane_id();
    const bool v = i < nl + nh;
    const uint64_t slot = !v ? 0ull : (i < nh ? kQHead + n - 1 - i : kQHead + (i - nh));
    const uint32_t unit = v ? q[slot] : 0u;
    const uint64_t k = v ? (in_len[unit] + kWvWin - 1) / kWvWin : 0ull;  // >= 1 (P > 0)
    const uint64_t r = wave_reserve(q_tiles(q), (v && k <= cap) ? k : 0ull);
    if (!v) continue;
    const uint64_t base = k <= cap ? r : cap;
    if (base + k <= cap) {
        for (uint64_t j = 0; j < k; ++j) {
            e[base + j].unit = unit;
            e[base + j].first = (uint32_t)base;
        }
        q[slot] = (uint32_t)base;  // the list entry now names the unit's first window (resolve pass)
    } else {
        for (uint64_t j = base; j < cap; ++j) e[j].unit = kTileSkip;  // reserved past the end: unused
        q[serial_off(n) + atomicAdd(q + 5, 1u)] = unit;  // the serial list
        q[slot] = kTileSkip;
    }
    }
}

__global__ __launch_bounds__(kWvBlock) void window_spec_kernel(const uint8_t* __restrict__ in,
                                                               const uint64_t* __restrict__ in_off,
                                                               const uint64_t* __restrict__ in_len, uint32_t n,
                                                               uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint8_t pk_all[kWvWaves * kWvPk];
    __shared__ __attribute__((aligned(16))) uint8_t mk_all[kWvWaves * kWvWin];
    const uint64_t T = min((uint64_t)*q_tiles(q), win_cap(n));
    if ((uint64_t)blockIdx.x * kWvWaves >= T) return;  // block-uniform
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* const pk = pk_all + wave * kWvPk;
    uint8_t* const mk = mk_all + wave * kWvWin;
    WinEnt* const tab = win_tab(q, n);
    const uint64_t G = (uint64_t)gridDim.x * kWvWaves;
    for (uint64_t g = (uint64_t)blockIdx.x * kWvWaves + wave; g < T; g += G) {
        WinEnt* const e = tab + g;
        const uint32_t unit = __builtin_amdgcn_readfirstlane(e->unit);
        if (unit == kTileSkip) continue;
        const uint64_t X = (g - __builtin_amdgcn_readfirstlane(e->first)) * (uint64_t)kWvWin;
        const WvWin w = wv_stage(pk, mk, in + in_off[unit], in_len[unit], X, lane);
        uint32_t ent, cs, ce;
        const uint32_t xw = wv_resolve(pk, mk, w, 0, lane, ent, cs, ce);
        const uint32_t words = wv_count(pk, w.sh, ent, ce);
        const uint32_t incl = wave_incl_sum(words, lane);
        const uint32_t total = readlane(incl, kWave - 1);
        // words before each verified record start of lanes 0 and 1 (window bytes [0, lim))
        const uint32_t lim = readlane(ce, 1);   // <= 2 * 73 bytes
        const uint32_t x1 = readlane(ent, 2);   // where the chain leaves lane 1's chunk
        const uint32_t w01 = readlane(incl, 1); // words of lanes 0 and 1
        uint16_t* const pre = reinterpret_cast<uint16_t*>(mk);  // the marks are dead by now
        wave_lds_sync();
        for (uint32_t i = lane; i < lim; i += kWave) pre[i] = 0xFFFFu;
        wave_lds_sync();
        if (lane < 2) {
            uint32_t ws = incl - words;
            for (uint32_t r = ent; r < ce;) {
                uint32_t t = pk[w.sh + r];
                uint32_t b1 = pk[w.sh + r + 1];
                uint32_t c9 = pk[w.sh + r + 9];
                asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));
                pre[r] = (uint16_t)min(ws, 0xFFFEu);
                ws += 1u + ((t == 0u) ? b1 : 0u) + ((t == 0xFFu) ? c9 : 0u);
                r += wv_len(t, c9);
            }
        }
        wave_lds_sync();
        // entry d = lane: walk until the chain meets a verified record start
        uint32_t r = lane, wd = 0;
        int32_t delta = 0;
        bool valid = false;
        for (;;) {
            if (r >= lim) {  // left lanes 0/1 uncoupled: valid only where the verified chain leaves
                valid = r == x1 && x1 != kEOFX;
                delta = (int32_t)wd - (int32_t)w01;
                break;
            }
            const uint32_t p = pre[r];
            if (p != 0xFFFFu) {
                valid = true;
                delta = (int32_t)wd - (int32_t)p;
                break;
            }
            uint32_t t = pk[w.sh + r];
            uint32_t b1 = pk[w.sh + r + 1];
            uint32_t c9 = pk[w.sh + r + 9];
            asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));
            const uint32_t len = wv_len(t, c9);
            if (r + len > w.rem) {  // message.zig:152-191: the record runs past the input
                valid = true;
                delta = kDeltaEof;
                break;
            }
            wd += 1u + ((t == 0u) ? b1 : 0u) + ((t == 0xFFu) ? c9 : 0u);
            r += len;
        }
        if (delta != kDeltaEof && (delta < -32767 || delta > 32767)) valid = false;
        const uint64_t vm = __ballot(valid);
        e->delta[lane] = (int16_t)(valid ? delta : 0);
        if (lane == 0) {
            e->exit = xw;
            e->total = total;
            e->valid = vm;
            e->ent = kWinNone;
        }
    }
}

__global__ __launch_bounds__(kWvBlock) void window_resolve_kernel(const uint8_t* __restrict__ in,
                                                                  const uint64_t* __restrict__ in_off,
                                                                  const uint64_t* __restrict__ in_len, uint32_t n,
                                                                  const uint64_t* __restrict__ out_cap,
                                                                  uint64_t* __restrict__ out_len,
                                                                  int32_t* __restrict__ status, uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint8_t pk_all[kWvWaves * kWvPk];
    __shared__ __attribute__((aligned(16))) uint8_t mk_all[kWvWaves * kWvWin];
    __shared__ int16_t dl_all[kWvWaves][kWinBatch][kWinD];
    const uint32_t nlist = q[0] + q[2];
    if ((uint64_t)blockIdx.x * kWvWaves >= nlist) return;  // block-uniform
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* const pk = pk_all + wave * kWvPk;
    uint8_t* const mk = mk_all + wave * kWvWin;
    WinEnt* const tab = win_tab(q, n);
    const uint32_t G = gridDim.x * kWvWaves;
    // a wave per listed long unit: the list entry names its first window (long_windows_kernel)
    for (uint32_t li = blockIdx.x * kWvWaves + wave; li < nlist; li += G) {
        {
            const uint32_t nh = q[2];
            const uint32_t b0 = q[li < nh ? kQHead + n - 1 - li : kQHead + (li - nh)];
            if (b0 == kTileSkip) continue;  // the serial decoder's
            const uint64_t g0 = b0;
            const uint32_t unit = __builtin_amdgcn_readfirstlane(tab[g0].unit);
            const uint8_t* const src = in + in_off[unit];
            const uint64_t P = in_len[unit];
            const uint64_t k = (P + kWvWin - 1) / kWvWin;
            uint64_t E = 0;     // the chain's next record start (unit-relative)
            uint64_t wacc = 0;  // output words so far
            int32_t st = ST_OK;
            for (uint64_t jb = 0; jb < k && st == ST_OK && E < P; jb += kWinBatch) {
                const uint32_t kb = (uint32_t)min((uint64_t)kWinBatch, k - jb);
                // the batch's exits, totals and valid masks (lane i: window jb + i) and deltas (LDS)
                uint32_t hx = 0, ht = 0, hvl = 0, hvh = 0;
                if (lane < kb) {
                    const WinEnt* const e = tab + g0 + jb + lane;
                    hx = e->exit;
                    ht = e->total;
                    const uint64_t v = e->valid;
                    hvl = (uint32_t)v;
                    hvh = (uint32_t)(v >> 32);
                }
                wave_lds_sync();
                for (uint32_t i = 0; i < kb; ++i) dl_all[wave][i][lane] = tab[g0 + jb + i].delta[lane];
                wave_lds_sync();
                uint32_t rent = kWinNone;  // lane i: the resolved entry of window jb + i
                uint64_t rwb = 0;
                for (uint32_t i = 0; i < kb; ++i) {  // wave-uniform
                    const uint64_t X = (jb + i) * (uint64_t)kWvWin;
                    if (E >= P) break;  // the unit's records are all resolved (E == P)
                    const uint32_t d = (uint32_t)(E - X);
                    const uint64_t vv = (uint64_t)readlane(hvl, i) | ((uint64_t)readlane(hvh, i) << 32);
                    uint32_t xw, words;
                    if (d < kWinD && ((vv >> d) & 1)) {
                        const int32_t dl = dl_all[wave][i][d];
                        xw = readlane(hx, i);
                        if (dl == kDeltaEof || xw == kEOFX) {
                            st = ST_EOF;
                            break;
                        }
                        words = (uint32_t)((int32_t)readlane(ht, i) + dl);
                    } else {  // stage the window again and resolve it from entry d
                        const WvWin w = wv_stage(pk, mk, src, P, X, lane);
                        uint32_t ent, cs, ce;
                        xw = wv_resolve(pk, mk, w, d, lane, ent, cs, ce);
                        if (xw == kEOFX) {
                            st = ST_EOF;
                            break;
                        }
                        const uint32_t wl = wv_count(pk, w.sh, ent, ce);
                        words = readlane(wave_incl_sum(wl, lane), kWave - 1);
                    }
                    if (lane == i) {
                        rent = d;
                        rwb = wacc;
                    }
                    wacc += words;
                    E = X + xw;
                }
                if (lane < kb) {
                    WinEnt* const e = tab + g0 + jb + lane;
                    e->ent = rent;
                    e->wb = rwb;
                }
            }
            if (lane == 0) {  // out_cap null: the size pass (estimateUnpackedSize)
                const uint64_t U = 8 * wacc;
                out_len[unit] = st == ST_OK ? U : 0;
                status[unit] = st != ST_OK ? st : (out_cap && U > out_cap[unit] ? ST_SPACE : ST_OK);
            }
        }
    }
}

__global__ __launch_bounds__(kWvBlock) void window_fill_kernel(const uint8_t* __restrict__ in,
                                                               const uint64_t* __restrict__ in_off,
                                                               const uint64_t* __restrict__ in_len, uint32_t n,
                                                               uint8_t* __restrict__ out,
                                                               const uint64_t* __restrict__ out_off,
                                                               const int32_t* __restrict__ status, uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint8_t pk_all[kWvWaves * kWvPk];
    __shared__ __attribute__((aligned(16))) uint8_t mk_all[kWvWaves * kWvWin];
    __shared__ uint64_t lut[256];  // tag -> v_perm selector that scatters the packed bytes
    const uint64_t T = min((uint64_t)*q_tiles(q), win_cap(n));
    if ((uint64_t)blockIdx.x * kWvWaves >= T) return;  // block-uniform
    lut[threadIdx.x] = expand_selector(threadIdx.x);
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* const pk = pk_all + wave * kWvPk;
    uint8_t* const mk = mk_all + wave * kWvWin;
    const WinEnt* const tab = win_tab(q, n);
    const uint64_t G = (uint64_t)gridDim.x * kWvWaves;
    for (uint64_t g = (uint64_t)blockIdx.x * kWvWaves + wave; g < T; g += G) {
        const WinEnt* const e = tab + g;
        const uint32_t unit = __builtin_amdgcn_readfirstlane(e->unit);
        if (unit == kTileSkip) continue;
        const uint32_t d = __builtin_amdgcn_readfirstlane(e->ent);
        if (d == kWinNone || status[unit] != ST_OK) continue;  // nothing to expand, or a failed unit
        const uint64_t X = (g - __builtin_amdgcn_readfirstlane(e->first)) * (uint64_t)kWvWin;
        const uint64_t wb = e->wb;
        const WvWin w = wv_stage(pk, mk, in + in_off[unit], in_len[unit], X, lane);
        uint32_t ent, cs, ce;
        (void)wv_resolve(pk, mk, w, d, lane, ent, cs, ce);
        const uint32_t words = wv_count(pk, w.sh, ent, ce);
        const uint32_t incl = wave_incl_sum(words, lane);
        const uint32_t total = readlane(incl, kWave - 1);
        uint64_t* const dst = reinterpret_cast<uint64_t*>(out + out_off[unit]) + wb;
        wv_expand(pk, mk, lut, w, ent, ce, incl - words, incl, total, dst, lane);
    }
}

// ---- small units, streaming encoder (round 4) -----------------------------
// Lane per unit, 64 units per wave in lockstep rounds of 8 words: round k's 64-B blocks of
// the wave's units come in by quad-coalesced 16-B loads issued a round ahead (only pieces
// inside the unit, temporal: the lane-streaming kernel below re-fetched lines its lanes had
// read, 4.2x its input; this one reads 3.6x, the neighbours of a unit's first and last lines
// being other bins' units), land in the
// units' 64-B LDS rings, and each lane codes its unit's 8 words with the Zig encoder's word
// step (message.zig:200-271; the small kernel's predicated state machine: a zero run is
// emitted when it ends, a literal run's count byte patched when it ends). A step completes at
// most one 16-B output chunk, which the lane stores at once (counted global stores); a chunk
// completed in one round sits next to its neighbours of the previous one, so lines fill up in
// L2 within a round or two. The small units come binned by length (<= 8, 16, 32, 64 words:
// 1, 2, 4 or 8 rounds; unit_class<4>), so a wave's units take about as many rounds.
constexpr uint32_t kEsWaves = 4;
constexpr uint32_t kEsBins = 4;   // small-unit bins of unit_class<4>: mid list bins 4 .. 7
constexpr uint32_t kEsRing = 80;  // ring row per unit: 64 B + 16 B pad (spreads the lanes' banks)

// AS1 (global) byte / 16-B stores: generic pointers would make FLAT instructions, which also
// count on lgkmcnt (every LDS wait of the loop would wait for them).
__device__ __forceinline__ void es_store16(uint8_t* p, uint64_t x0, uint64_t x1) {
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p),
                 "v"(u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)})
                 : "memory");
}
__device__ __forceinline__ void es_store_byte(uint8_t* p, uint32_t v) {
    *reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(reinterpret_cast<uintptr_t>(p)) = (uint8_t)v;
}
// bytes [lo, hi) of a 16-B chunk at c16 (x0 = bytes 0-7, x1 = 8-15), global stores
__device__ __forceinline__ void es_store_partial16(uint8_t* c16, uint32_t lo, uint32_t hi, uint64_t x0, uint64_t x1) {
    typedef __attribute__((address_space(1))) uint8_t g8;
    typedef __attribute__((address_space(1))) uint16_t g16;
    typedef __attribute__((address_space(1))) uint32_t g32;
    typedef __attribute__((address_space(1))) uint64_t g64;
    const uintptr_t base = reinterpret_cast<uintptr_t>(c16);
    auto put = [&](uint32_t sz) {  // bytes [lo, lo + sz), lo aligned to sz
        const uint64_t v = lo < 8 ? x0 >> (8 * lo) : x1 >> (8 * (lo - 8));
        const uintptr_t p = base + lo;
        if (sz == 8) *reinterpret_cast<g64*>(p) = v;
        else if (sz == 4) *reinterpret_cast<g32*>(p) = (uint32_t)v;
        else if (sz == 2) *reinterpret_cast<g16*>(p) = (uint16_t)v;
        else *reinterpret_cast<g8*>(p) = (uint8_t)v;
        lo += sz;
    };
    if ((lo & 1) && lo + 1 <= hi) put(1);
    if ((lo & 2) && lo + 2 <= hi) put(2);
    if ((lo & 4) && lo + 4 <= hi) put(4);
    if (lo + 8 <= hi) put(8);
    if (lo + 4 <= hi) put(4);
    if (lo + 2 <= hi) put(2);
    if (lo + 1 <= hi) put(1);
}

template <bool WRITE>
__global__ __launch_bounds__(kEsWaves * kWave) void encode_stream_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ in_len,
    uint32_t n, uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
    const uint64_t* __restrict__ out_cap, uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
    const uint32_t* __restrict__ q) {
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    __shared__ __attribute__((aligned(16))) uint8_t ring_blk[kEsWaves * kWave * kEsRing];
    if (WRITE)
        for (uint32_t t = threadIdx.x; t < 256; t += kEsWaves * kWave) lut[t] = compact_selector(t);
    __syncthreads();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* const ring_all = ring_blk + wave * (kWave * kEsRing);
    const uint32_t lane = lane_id();
    // the small units: mid-list bins 4 .. 7 (unit_class<4>)
    const uint32_t b0i = q[11 + CL_MID_BINS - kEsBins];
    const uint32_t count = q[4] - b0i;
    const uint32_t* const list = q + kQHead + 2ull * n + b0i;
    const uint32_t wv = blockIdx.x * kEsWaves + wave;
    if (wv * kWave >= count) return;  // wave-uniform
    const uint32_t slot = wv * kWave + lane;
    const bool valid = slot < count;
    const uint32_t unit = valid ? list[slot] : 0u;

    // ---- per-lane unit ---------------------------------------------------------------
    const uint8_t* src = cpk_dummy16;
    uint64_t len = 0, cap = 0;
    uint8_t* dst = out;
    int32_t st = ST_OK;
    if (valid) {
        src = in + in_off[unit];
        len = in_len[unit];
        if (reinterpret_cast<uintptr_t>(src) & 7) st = ST_ARG;
        else if (len & 7) st = ST_SIZE;  // message.zig:201
        if (WRITE) {
            dst = out + out_off[unit];
            cap = out_cap[unit];
        }
    }
    const bool take = valid && st == ST_OK && len > 0;
    if (!take) src = cpk_dummy16;
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);  // 0 or 8
    const uint32_t s8 = s >> 3;
    const uint32_t nw = take ? s8 + (uint32_t)(len >> 3) : 0u;  // aligned-space word end (<= 65 words)
    const uint32_t nr = (nw + 7) >> 3;                            // rounds of this unit
    const uint32_t npieces = take ? (s + (uint32_t)len + 15) >> 4 : 0u;
    const uint32_t maxr = __builtin_amdgcn_readfirstlane(wave_max_u32(nr));

    const uint4* qsrc[4];
    uint32_t qlast[4];
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m) {
        const uint32_t r = 16 * m + lane / 4;
        const uint64_t rb = __shfl(reinterpret_cast<uint64_t>(src - s), r, kWave);
        const uint32_t rn = __shfl(npieces, r, kWave);
        qsrc[m] = reinterpret_cast<const uint4*>(rn ? reinterpret_cast<const uint8_t*>(rb) : cpk_dummy16);
        qlast[m] = rn ? rn - 1 : 0u;
    }
    const uint32_t qp = lane & 3;
    u32x4 d0, d1, d2, d3;
    // only pieces inside the unit are loaded (a lane past its unit's last piece skips the
    // load: the ring keeps stale bytes the steps never read), and with the temporal hint, so a
    // line read for one round is still in L2 for the next (round 4: clamped non-temporal
    // re-loads of the last piece read 656 MB per C5 launch, 4.8x the small units' input)
    auto load = [&](uint32_t k) {
        if (4 * k + qp <= qlast[0]) ds_gload16(d0, qsrc[0] + 4 * k + qp);
        if (4 * k + qp <= qlast[1]) ds_gload16(d1, qsrc[1] + 4 * k + qp);
        if (4 * k + qp <= qlast[2]) ds_gload16(d2, qsrc[2] + 4 * k + qp);
        if (4 * k + qp <= qlast[3]) ds_gload16(d3, qsrc[3] + 4 * k + qp);
    };
    uint8_t* const wq = ring_all + (lane / 4) * kEsRing + 16 * qp;  // unit 16m + l/4: + 16 * kEsRing * m
    const uint64_t* const ring = reinterpret_cast<const uint64_t*>(ring_all + lane * kEsRing);

    // ---- the encoder's state (encode_small_kernel's word step) ---------------------------
    const uint32_t da = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15);
    uint8_t* const db = dst - da;  // 16-B aligned base of the output slot
    uint64_t op = 0;               // packed bytes so far
    uint64_t b0 = 0, b1 = 0;       // the output chunk being assembled: chunk (da + op) >> 4
    uint32_t mode = 0, run = 0;    // 0: none, 1: zero run, 2: literal run; its length
    uint64_t cpos = 0;             // literal run: output offset of its count byte
    uint64_t f0 = 0, f1 = 0, fch = 0;  // a chunk the step completed
    bool fpend = false;
    const uint64_t lim = cap > ~0ull - 16 ? ~0ull : da + cap;  // slot end (saturated)
    auto app = [&](bool p, uint64_t v, uint32_t nb) {  // append nb <= 8 bytes of v when p
        if (WRITE) {
            const uint32_t k = (uint32_t)((da + op) & 15);
            const uint32_t sh = 8 * (k & 7);
            const uint64_t lo = v << sh, hi = (v >> 1) >> (63 - sh);
            const bool low = k < 8;
            if (p) {
                b0 |= low ? lo : 0ull;
                b1 |= low ? hi : lo;
            }
            if (p && k + nb >= 16) {
                f0 = b0;
                f1 = b1;
                fch = (da + op) >> 4;
                fpend = true;
                b0 = hi;
                b1 = 0;
            }
        }
        op += p ? nb : 0u;
    };
    auto patch = [&](bool p, uint32_t c) {  // the open literal run's count byte = c
        if (!WRITE || !p) return;
        const uint64_t x = da + cpos;
        const uint32_t k = (uint32_t)(x & 15);
        const uint64_t m0 = k < 8 ? (uint64_t)c << (8 * k) : 0ull, m1 = k < 8 ? 0ull : (uint64_t)c << (8 * (k - 8));
        if ((x >> 4) == ((da + op) >> 4)) {
            b0 |= m0;
            b1 |= m1;
        } else if (fpend && (x >> 4) == fch) {
            f0 |= m0;
            f1 |= m1;
        } else if (cpos < cap) {
            es_store_byte(db + x, c);  // after the chunk's store (same wave, same address)
        }
    };
    auto step = [&](uint64_t w, bool vw) {  // message.zig:206-266, one word
        const uint32_t tg = nonzero_tag(w);
        const bool isz = tg == 0u, isf = tg == 0xFFu;
        const bool cz = vw && mode == 1 && isz && run < 256;
        const bool cf = vw && mode == 2 && isf && run < 256;
        const bool cl = vw && mode != 0 && !cz && !cf;
        app(cl && mode == 1, (uint64_t)(run - 1) << 8, 2);  // 00 <count>
        patch(cl && mode == 2, run - 1);
        const bool nzr = vw && !cz && !cf && isz;
        const bool nfr = vw && !cz && !cf && isf;
        const bool mx = vw && !isz && !isf;
        const uint64_t v = cf ? w : (nfr ? (0xFFull | (w << 8)) : ((uint64_t)tg | (WRITE ? perm64(w, lut[tg]) : 0ull)));
        app(cf || nfr || mx, v, (cf || nfr) ? 8u : 1u + __popc(tg));
        app(nfr, w >> 56, 2);  // w7, then the count byte (0 until patched)
        cpos = nfr ? op - 1 : cpos;
        mode = (cz || nzr) ? 1u : ((cf || nfr) ? 2u : (vw ? 0u : mode));
        run = (cz || cf) ? run + 1 : ((nzr || nfr) ? 1u : run);
    };
    uint32_t younger = 0;  // stores issued after the round's loads (counted ones)
    // a completed chunk: one 16-B store when it lies inside the slot, else its slot bytes
    auto flush_pending = [&]() {
        if (!WRITE) return;
        const bool full = fpend && 16 * fch >= da && 16 * fch + 16 <= lim;
        if (__builtin_amdgcn_ballot_w64(full) != 0) {
            if (full) es_store16(db + 16 * fch, f0, f1);
            ++younger;
        }
        if (fpend && !full) {  // the slot's first chunk, or one past its capacity
            const uint64_t cs = 16 * fch;
            const uint64_t a = max(cs, (uint64_t)da), e = min(cs + 16, lim);
            if (a < e) es_store_partial16(db + cs, (uint32_t)(a - cs), (uint32_t)(e - cs), f0, f1);
        }
        fpend = false;
    };

    if (maxr > 0) load(0);
    for (uint32_t k = 0; k < maxr; ++k) {
        vmcnt_at_most63(younger);  // round k's loads have landed
        asm volatile("" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
        younger = 0;
        wave_lds_sync();  // every lane is done with round k-1's ring reads
        *reinterpret_cast<u32x4*>(wq) = d0;
        *reinterpret_cast<u32x4*>(wq + 16 * kEsRing) = d1;
        *reinterpret_cast<u32x4*>(wq + 32 * kEsRing) = d2;
        *reinterpret_cast<u32x4*>(wq + 48 * kEsRing) = d3;
        if (k + 1 < maxr) load(k + 1);
        wave_lds_sync();
#pragma unroll 2
        for (uint32_t t = 0; t < 8; ++t) {
            const uint32_t aw = 8 * k + t;
            step(ring[t], take && aw >= s8 && aw < nw);
            flush_pending();
        }
        if (take && k + 1 == nr) {  // the unit ends in this round
            app(mode == 1, (uint64_t)(run - 1) << 8, 2);  // inside a run
            patch(mode == 2, run - 1);
            mode = 0;
        }
        flush_pending();
        if (take && k + 1 == nr && WRITE && ((da + op) & 15)) {  // the last, partial chunk
            const uint64_t cs = ((da + op) >> 4) << 4;
            const uint64_t a = max(cs, (uint64_t)da), e = min(da + op, lim);
            if (a < e) es_store_partial16(db + cs, (uint32_t)(a - cs), (uint32_t)(e - cs), b0, b1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!valid) return;
    out_len[unit] = st == ST_OK ? op : 0;
    status[unit] = st != ST_OK ? st : ((WRITE && op > cap) ? ST_SPACE : ST_OK);
}


// ---- small units, lane per unit ----------------------------------------------------------
// (a lane-per-unit encode_small_kernel, removed in round 5 (at 869fccf), measured C5 encode
// 0.630 ms against the streaming encoder's 0.588-0.603, same box)
// A persistent grid: each wave owns a contiguous range of the small list and its lanes
// take the range's next unit as they finish (a wave-uniform cursor, as in
// validate_kernel), so one longer unit does not idle the rest of its wave. Every turn
// of the wave's loop issues at most one read per lane (the unit's metadata, or its next
// 16 B) and then codes the 16 B read one turn earlier: the read's latency overlaps the
// work.
constexpr uint32_t kSmBlock = 256;
enum : uint32_t { SM_IDLE, SM_EXIT, SM_META, SM_FIRST, SM_RUN };



// unpackPacked (message.zig:88-145) for one unit per lane. Each lane keeps a 64-B ring of
// its unit's packed bytes in LDS (piece p at slot p % 4). A turn codes the records that
// start in the lane's 32-B span [16k, 16k + 32) -- one record per loop pass on every lane,
// predicated (no per-record branches: zero-run and literal-run records take the same path
// as the others, a literal word as if it followed an FF tag) -- while later pieces are in
// flight into registers: every other turn the next four (64 B) are loaded at once, and they
// enter the ring two at a time at the start of the next two turns.
// A truncated record is UnexpectedEof with nothing more written.
// Output (round 3): lanes write to different units, so a lane's own 16-B store is a memory
// transaction of its own, and those scattered partial-line writes also slowed every kernel
// beside this one. Each lane stages its words in LDS by absolutely aligned
// 64-B chunks; after each record pass the wave stores the chunks completed in it, a quad of
// lanes per chunk (16 chunks of 64 contiguous bytes per store instruction). A unit's partial
// first and last chunks, and chunks a zero run completes, are stored by their lane.
constexpr uint32_t kSdRing = 80;  // LDS bytes per lane: the 64-B ring + 16 B (fewer bank conflicts)
constexpr uint32_t kSdChunk = 8;         // output words per staged chunk (64 B)
constexpr uint32_t kSdGroup = 2 * kWave / kSdChunk; // chunks per cooperative store instruction
__global__ __launch_bounds__(kSmBlock) void decode_small_kernel(const uint8_t* __restrict__ in,
                                                                const uint64_t* __restrict__ in_off,
                                                                const uint64_t* __restrict__ in_len, uint32_t n,
                                                                uint8_t* __restrict__ out,
                                                                const uint64_t* __restrict__ out_off,
                                                                const uint64_t* __restrict__ out_cap,
                                                                uint64_t* __restrict__ out_len,
                                                                int32_t* __restrict__ status, const uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[kSmBlock * kSdRing];
    // each lane's output words by absolutely aligned 8-word (64-B) chunks; a full chunk is
    // stored by a quad of the wave (4 x 16 B), 16 chunks per store instruction
    __shared__ __attribute__((aligned(16))) uint64_t ostage_all[kSmBlock * kSdChunk];
    __shared__ __attribute__((aligned(16))) uint64_t ctab_all[(kSmBlock / kWave) * kSdGroup * 2];
    uint64_t* const ostage = ostage_all + threadIdx.x * kSdChunk;
    uint64_t* const ctab = ctab_all + (threadIdx.x >> 6) * (2 * kSdGroup);
    const uint32_t wbase_t = threadIdx.x & ~(kWave - 1);
    lut[threadIdx.x] = expand_selector(threadIdx.x);
    __syncthreads();
    const uint32_t count = q[3];
    const uint32_t* const list = q + kQHead + n;
    const uint32_t lane = lane_id();
    const uint32_t gw = blockIdx.x * (kSmBlock / kWave) + (threadIdx.x >> 6);
    const uint32_t GW = gridDim.x * (kSmBlock / kWave);
    const uint32_t per = (count + GW - 1) / GW;
    const uint64_t first = (uint64_t)gw * per;
    const uint64_t last = min((uint64_t)count, first + per);
    uint64_t cursor = first;  // wave-uniform
    uint8_t* const ring = ring_all + threadIdx.x * kSdRing;

    uint32_t kind = SM_IDLE, unit = 0;
    const uint8_t* base = in;  // 16-B aligned base of the packed unit
    uint32_t end = 0, pos = 0, k = 0, np = 0, lit = 0;  // aligned space: bytes [s, end); span start piece
    uint4 d0, d1, d2, d3;                                // pieces in flight
    uint64_t* dst = nullptr;
    uint32_t capw = 0, wo = 0;
    uint64_t cap = 0;

    constexpr uint32_t SW = kSdChunk;
    uint32_t ph = 0;      // the slot's first word's position in its aligned chunk
    bool rdy = false;     // a full chunk waits for the wave's flush
    uint64_t* rdst = nullptr;
    // the lane itself stores the staged words [lo, hi] (slot word indices) of the chunk ending at e
    auto flush = [&](uint32_t e, uint32_t lo, uint32_t hi) {
        const int32_t cb = (int32_t)e - (int32_t)(SW - 1);
#pragma unroll
        for (uint32_t pp = 0; pp < SW / 2; ++pp) {
            const int32_t w0 = cb + 2 * (int32_t)pp, w1 = w0 + 1;
            const bool v0 = w0 >= (int32_t)lo && w0 <= (int32_t)hi, v1 = w1 >= (int32_t)lo && w1 <= (int32_t)hi;
            if (v0 | v1) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(ostage + 2 * pp);
                if (v0 && v1) *reinterpret_cast<u32x4*>(dst + w0) = v;
                else if (v0) dst[w0] = (uint64_t)v.x | ((uint64_t)v.y << 32);
                else dst[w1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
            }
        }
    };
    // word w of the slot, staged at its chunk position; a full chunk is left to the wave's
    // flush when `defer` (nothing else is staged by this lane before it), else stored at once
    auto put = [&](uint32_t w, uint64_t word, bool defer) {
        if (w < capw) {
            const uint32_t j = (ph + w) & (SW - 1);
            ostage[j] = word;
            if (j == SW - 1) {
                if (defer && w >= SW - 1) {
                    rdy = true;
                    rdst = dst + (w - (SW - 1));
                } else {
                    flush(w, w >= SW - 1 ? w - (SW - 1) : 0u, w);
                }
            }
        }
    };
    auto finish = [&](int32_t st) {
        if (st == ST_OK) {
            out_len[unit] = 8ull * wo;
            status[unit] = 8ull * wo > cap ? ST_SPACE : ST_OK;
        } else {
            out_len[unit] = 0;
            status[unit] = st;
        }
        kind = SM_IDLE;
    };
    auto ld = [&](uint32_t i) { return *reinterpret_cast<const uint4*>(base + 16ull * min(i, np - 1)); };

    // The metadata of the wave's next 64 list entries, one per lane (lane i: entry cb + i),
    // loaded together when the cursor leaves the cached block: a lane taking a unit gets its
    // offsets by shuffles in the same turn (no dependent load and no stall of the whole wave
    // per new unit), and the four arrays' lines are read once, not once per taking lane.
    uint64_t cb = first;  // wave-uniform
    uint32_t c_unit = 0;
    uint64_t c_off = 0, c_len = 0, c_oo = 0, c_cap = 0;
    auto fill_cache = [&](uint64_t b) {
        cb = b;
        const uint64_t e = b + lane;
        if (e < last) {
            c_unit = list[e];
            c_off = in_off[c_unit];
            c_len = in_len[c_unit];
            c_oo = out_off[c_unit];
            c_cap = out_cap[c_unit];
        }
    };
    if (first < last) fill_cache(first);
    uint32_t cslot = 0;  // a SM_META lane's cache lane
    for (;;) {
        const uint64_t idle = __ballot(kind == SM_IDLE);
        if (idle) {
            if (cursor < last) {
                if (cursor >= cb + kWave) fill_cache(cursor);  // wave-uniform
                const uint64_t avail = min(last, cb + kWave) - cursor;  // cached entries from the cursor
                const uint64_t rank = __popcll(idle & ((1ull << lane) - 1ull));
                if (kind == SM_IDLE) {
                    if (rank < avail) {
                        cslot = (uint32_t)(cursor - cb + rank);
                        kind = SM_META;
                    } else if (cursor + rank >= last) {
                        kind = SM_EXIT;
                    }  // else: a unit from the next block, next turn
                }
                cursor += min((uint64_t)__popcll(idle), avail);
            } else if (kind == SM_IDLE) {
                kind = SM_EXIT;
            }
        }
        if (__ballot(kind != SM_EXIT) == 0) break;
        // ---- this turn's reads (and last turn's pieces into the ring) -------------------
        uint64_t m_off = 0, m_len = 0, m_oo = 0, m_cap = 0;
        if (__ballot(kind == SM_META) != 0) {  // every lane shuffles (a taker reads its cache lane)
            const uint32_t src_l = kind == SM_META ? cslot : lane;
            const uint32_t u = (uint32_t)__shfl((int)c_unit, (int)src_l, kWave);
            m_off = shfl_u64(c_off, src_l);
            m_len = shfl_u64(c_len, src_l);
            m_oo = shfl_u64(c_oo, src_l);
            m_cap = shfl_u64(c_cap, src_l);
            if (kind == SM_META) unit = u;
        }
        // a new unit is set up from its metadata and issues its first loads in the same turn
        if (kind == SM_META) {
            const uint8_t* const src = in + m_off;
            const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
            base = src - s;
            end = s + (uint32_t)m_len;  // m_len <= kSmDecP
            np = (end + 15) >> 4;
            pos = s;
            k = 0;
            lit = 0;
            uint8_t* const o = out + m_oo;
            dst = reinterpret_cast<uint64_t*>(o);
            cap = m_cap;
            capw = (uint32_t)(m_cap >> 3);
            wo = 0;
            ph = (uint32_t)(reinterpret_cast<uintptr_t>(o) >> 3) & (SW - 1);
            if (m_len == 0) finish(ST_OK);  // an empty unit writes nothing: any slot will do
            else if (reinterpret_cast<uintptr_t>(o) & 7) finish(ST_ARG);
            else kind = SM_FIRST;
        }
        if (kind == SM_FIRST) {
            d0 = ld(0);
            d1 = ld(1);
            d2 = ld(2);
            d3 = ld(3);
        } else if (kind == SM_RUN) {
            // pieces k+2, k+3 enter the ring; every other turn (k = 0 mod 4) the next four
            // pieces are loaded together (64 contiguous bytes: a line's half is fetched in one
            // burst, not 16 B a turn while other lanes' traffic evicts it in between)
            uint4* const r4 = reinterpret_cast<uint4*>(ring);
            if (k == 0) {
                r4[0] = d0;
                r4[1] = d1;
                r4[2] = d2;
                r4[3] = d3;
            } else if (k & 2) {
                r4[(k + 2) & 3] = d0;
                r4[(k + 3) & 3] = d1;
            } else {
                r4[(k + 2) & 3] = d2;
                r4[(k + 3) & 3] = d3;
            }
            if ((k & 2) == 0) {
                d0 = ld(k + 4);
                d1 = ld(k + 5);
                d2 = ld(k + 6);
                d3 = ld(k + 7);
            }
        }
        // ---- decode -------------------------------------------------------------------------
        bool act = kind == SM_RUN;  // the lanes that code this turn
        if (kind == SM_FIRST) {
            kind = SM_RUN;  // its first pieces enter the ring next turn
        }
        wave_lds_sync();  // the ring writes above are visible to the reads below
        const uint32_t lim = 16 * (k + 2);  // span end
        for (;;) {  // one record per lane per pass; predicated body, uniform exit
            const bool go = act && pos < lim && (lit != 0 || pos < end);
            if (__ballot(go) == 0) break;
            const bool isl = lit != 0;
            const uint32_t qq = isl ? pos - 1 : pos;  // a literal word reads as if after an FF tag at pos - 1
            uint32_t t = ring[pos & 63];
            uint32_t b1 = ring[(pos + 1) & 63];
            uint32_t c9 = ring[(pos + 9) & 63];
            const uint32_t a = (qq + 1) & ~7u;
            uint64_t lo = *reinterpret_cast<const uint64_t*>(ring + (a & 63));
            uint64_t hi = *reinterpret_cast<const uint64_t*>(ring + ((a + 8) & 63));
            asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9), "+v"(lo), "+v"(hi));  // one LDS round trip
            const uint32_t sh = ((qq + 1) & 7) * 8;
            const uint64_t pay = (lo >> sh) | ((hi << 1) << (63 - sh));  // bytes qq+1 .. qq+8
            const bool z = !isl && t == 0u, f = !isl && t == 0xFFu;
            // message.zig:101-141: 00 c -> c+1 zero words; FF w c -> w, then c literal words;
            // other tags -> popc(t) bytes scattered to the set bits
            const uint32_t len = isl ? 8u : 1u + __popc(t) + (uint32_t)(z | f);
            const bool eof = go && !isl && (pos + len > end || (f && pos + 10u + 8u * c9 > end));
            const bool ok = go && !eof;
            const uint64_t word = perm64(pay, lut[isl ? 0xFFu : t]);  // lut[0] = zero word
            // Output words are staged in LDS by aligned 64-B chunks (put); a word at capw or
            // beyond is not stored.
            const uint32_t zr = (ok && z) ? b1 : 0u;  // the zero run's further words
            if (ok) put(wo, word, zr == 0u);
            for (uint32_t j = 1; j <= zr; ++j) put(wo + j, 0ull, false);
            pos = ok ? pos + len : pos;
            lit = ok ? (isl ? lit - 1u : (f ? c9 : 0u)) : lit;
            wo = ok ? wo + 1u + zr : wo;
            if (eof) finish(ST_EOF);
            act = act && !eof;
            // the wave stores the full chunks of this pass: quad i takes the i-th ready lane's
            const uint64_t rm = __ballot(rdy);
            if (rm) {
                const uint32_t nr = (uint32_t)__popcll(rm);
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u));
                for (uint32_t g = 0; g < nr; g += kSdGroup) {
                    wave_lds_sync();
                    if (rdy && rank >= g && rank < g + kSdGroup) {
                        ctab[2 * (rank - g)] = reinterpret_cast<uint64_t>(rdst);
                        ctab[2 * (rank - g) + 1] = lane;
                    }
                    wave_lds_sync();
                    const uint32_t qd = lane / (kSdChunk / 2);  // the chunk this lane stores 16 B of
                    const uint32_t qi = lane % (kSdChunk / 2);
                    if (g + qd < nr) {
                        uint64_t* const cd = reinterpret_cast<uint64_t*>(ctab[2 * qd]);
                        const uint32_t sl = (uint32_t)ctab[2 * qd + 1];
                        const u32x4 v = *reinterpret_cast<const u32x4*>(ostage_all + (wbase_t + sl) * kSdChunk + 2 * qi);
                        *reinterpret_cast<u32x4*>(cd + 2 * qi) = v;
                    }
                }
                rdy = false;
            }
        }
        if (act) {  // still running: done, or the next span
            if (pos >= end && lit == 0) {
                // the last staged chunk, if its last word is not the chunk's last (a unit that
                // overran its slot stopped staging at word capw - 1)
                const uint32_t lw = min(wo, capw);  // words staged
                if (lw > 0 && ((ph + lw - 1u) & (SW - 1)) != SW - 1) {
                    const uint32_t e = lw - 1u + (SW - 1 - ((ph + lw - 1u) & (SW - 1)));
                    const uint32_t c0 = e + 1u >= SW ? e + 1u - SW : 0u;  // the chunk's first slot word
                    flush(e, c0, lw - 1u);
                }
                finish(ST_OK);
            } else {
                k += 2;
            }
        }
    }
}

// unpackPacked (message.zig:88-145) for small units, a GROUP of units per wave (round 3,
// DESIGN.md §2.6). decode_small_kernel's lanes each stream their own unit: every load and
// store of a wave goes to 64 different units, 16 B each, and the partly written lines those
// stores leave behind make HBM traffic 2-3x the bytes (C5 PMC: 428 MB written for ~130 MB of
// output). Here a wave takes up to 64 consecutive units of the small list whose packed pieces
// fit kSgP bytes of LDS and whose capacities fit kSgW words:
//   1. meta: lane i reads entry i's offsets / lengths (one coalesced load per array); wave
//      scans of the pieces and capacity words give each unit its LDS offsets;
//   2. load: the group's 16-B pieces, flattened (piece j -> its unit by a binary search of
//      the piece prefix in LDS), 64 per instruction, contiguous within each unit;
//   3. decode: lane i walks unit i's records from LDS (one record per pass on every lane,
//      predicated as decode_small_kernel), writing its words into its LDS output slot;
//   4. store: the OK units' words, flattened by 16-B pairs the same way, so the stores of a
//      wave write whole runs of each unit's slot.
// A unit is written only when it decodes OK within its capacity: small units are
// all-or-nothing too (message.zig:90 raises before any output), like mid and long units.
// Opt-in (capnp_packed_set_all_or_nothing(1)): measured slower than decode_small_kernel, because a group's
// decode phase waits for its longest unit (C5's sizes are heavy-tailed) while the lane
// kernel refills each lane as its unit ends.
constexpr uint32_t kSgWaves = 4;
constexpr uint32_t kSgP = 4096;   // packed bytes (16-B pieces, from each unit's aligned base) per group
constexpr uint32_t kSgW = 1024;   // output capacity words per group (8 KiB: any one small unit fits)
constexpr uint32_t kSgPad = 32;   // read slack past the last piece (a record's count byte, a word's tail)
static_assert(kSgW * 8 >= kSmDecCap && kSgP >= 16 * ((kSmDecP + 30) / 16), "one small unit fits a group");

// index of the last entry of the wave-ordered prefix table pfx[0..cnt) that is <= j
__device__ __forceinline__ uint32_t sg_find(const uint32_t* pfx, uint32_t cnt, uint32_t j) {
    uint32_t lo = 0, hi = cnt;  // pfx[lo] <= j < pfx[hi] (pfx[cnt] = +inf)
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        const uint32_t mid = (lo + hi) >> 1;
        const bool le = mid < cnt && pfx[mid] <= j;
        lo = (le && mid > lo) ? mid : lo;
        hi = (!le && mid < hi) ? mid : hi;
    }
    return lo;
}

__global__ __launch_bounds__(kSgWaves * kWave) void decode_small_group_kernel(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ in_len,
    uint32_t n, uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
    const uint64_t* __restrict__ out_cap, uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
    const uint32_t* q) {
    __shared__ __attribute__((aligned(16))) uint64_t lut[256];
    __shared__ __attribute__((aligned(16))) uint8_t pin_all[kSgWaves][kSgP + kSgPad];
    __shared__ __attribute__((aligned(16))) uint64_t pout_all[kSgWaves][kSgW];
    __shared__ uint32_t pfx_all[kSgWaves][2][kWave];  // exclusive prefix: pieces, output pairs
    for (uint32_t i = threadIdx.x; i < 256; i += kSgWaves * kWave) lut[i] = expand_selector(i);
    __syncthreads();
    const uint32_t count = q[3];
    const uint32_t* const list = q + kQHead + n;
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* const pin = pin_all[wave];
    uint64_t* const pout = pout_all[wave];
    uint32_t* const ppf = pfx_all[wave][0];
    uint32_t* const opf = pfx_all[wave][1];
    // a contiguous range of the small list per wave (batch order within the class)
    const uint32_t gw = blockIdx.x * kSgWaves + wave, GW = gridDim.x * kSgWaves;
    const uint32_t per = (count + GW - 1) / GW;
    uint64_t cursor = (uint64_t)gw * per;
    const uint64_t last = min((uint64_t)count, cursor + per);
    while (cursor < last) {  // wave-uniform
        // ---- 1. meta of the next (up to) 64 entries -----------------------------------------
        const bool valid = cursor + lane < last;
        uint32_t unit = 0, P = 0, s = 0, np = 0, capw = 0;
        uint64_t src = 0, dst = 0, cap = 0;
        if (valid) {
            unit = list[cursor + lane];
            const uint64_t off = in_off[unit];
            P = (uint32_t)in_len[unit];  // <= kSmDecP
            cap = out_cap[unit];         // <= kSmDecCap
            dst = reinterpret_cast<uint64_t>(out + out_off[unit]);
            src = reinterpret_cast<uint64_t>(in + off);
            s = (uint32_t)(src & 15);
            np = P ? (s + P + 15) >> 4 : 0u;
            capw = (uint32_t)(cap >> 3);
        }
        const uint32_t ip = wave_incl_sum(valid ? np : 0u, lane);
        const uint32_t iw = wave_incl_sum(valid ? capw : 0u, lane);
        const bool fits = valid && 16u * ip <= kSgP && iw <= kSgW;  // prefix-monotone
        const uint32_t g = (uint32_t)__popcll(__ballot(fits));     // >= 1: one small unit always fits
        const bool mine = lane < g;
        const uint32_t pb = ip - np, wb = iw - capw;  // this unit's first piece / output word
        const uint32_t NP = readlane(ip, g - 1);
        wave_lds_sync();  // the previous group's LDS reads are done
        ppf[lane] = mine ? pb : 0xFFFFFFFFu;
        wave_lds_sync();
        // ---- 2. load the group's pieces, flattened ------------------------------------------
        // piece j of the group: its unit k (binary search of the piece prefix), then 16 B from
        // the unit's aligned base (all lanes take part in the bpermutes; past NP they re-load
        // the last piece and store nothing)
        auto piece = [&](uint32_t j) {
            const uint32_t jj = j < NP ? j : NP - 1;
            const uint32_t k = sg_find(ppf, g, jj);
            const uint64_t base = (uint64_t)__shfl((long long)src, (int)k, kWave) & ~15ull;
            const uint32_t pk0 = (uint32_t)__shfl((int)pb, (int)k, kWave);
            return *reinterpret_cast<const uint4*>(base + 16ull * (jj - pk0));
        };
        for (uint32_t j0 = 0; j0 < NP; j0 += 2 * kWave) {  // two loads in flight per lane
            const uint32_t ja = j0 + lane, jb = j0 + kWave + lane;
            const uint4 va = piece(ja);
            const uint4 vb = piece(jb);
            if (ja < NP) *reinterpret_cast<uint4*>(pin + 16 * ja) = va;
            if (jb < NP) *reinterpret_cast<uint4*>(pin + 16 * jb) = vb;
        }
        wave_lds_sync();
        // ---- 3. decode: lane i walks unit i -------------------------------------------------
        const uint8_t* const b = pin + (mine ? 16 * pb : 0u);
        uint64_t* const o = pout + (mine ? wb : 0u);
        uint32_t pos = s, end = s + P, lit = 0, wo = 0;
        int32_t st = ST_OK;
        bool act = mine && P > 0;
        if (mine && P > 0 && (dst & 7)) {
            st = ST_ARG;
            act = false;
        }
        for (;;) {  // one record per lane per pass; predicated body, uniform exit
            const bool go = act && (lit != 0 || pos < end);
            if (__ballot(go) == 0) break;
            const bool isl = lit != 0;
            const uint32_t p0 = go ? pos : 0u;
            const uint32_t qq = isl ? p0 - 1 : p0;  // a literal word reads as if after an FF tag at pos - 1
            uint32_t t = b[p0];
            uint32_t b1 = b[p0 + 1];
            uint32_t c9 = b[p0 + 9];
            const uint32_t a = (qq + 1) & ~7u;
            uint64_t lo = *reinterpret_cast<const uint64_t*>(b + a);
            uint64_t hi = *reinterpret_cast<const uint64_t*>(b + a + 8);
            asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9), "+v"(lo), "+v"(hi));  // one LDS round trip
            const uint32_t sh = ((qq + 1) & 7) * 8;
            const uint64_t pay = (lo >> sh) | ((hi << 1) << (63 - sh));  // bytes qq+1 .. qq+8
            const bool z = !isl && t == 0u, f = !isl && t == 0xFFu;
            // message.zig:101-141: 00 c -> c+1 zero words; FF w c -> w, then c literal words;
            // other tags -> popc(t) bytes scattered to the set bits
            const uint32_t len = isl ? 8u : 1u + __popc(t) + (uint32_t)(z | f);
            const bool eof = go && !isl && (pos + len > end || (f && pos + 10u + 8u * c9 > end));
            const bool ok = go && !eof;
            const uint64_t word = perm64(pay, lut[isl ? 0xFFu : t]);  // lut[0] = zero word
            if (ok && wo < capw) o[wo] = word;
            const uint32_t zr = (ok && z) ? b1 : 0u;  // the zero run's further words
            for (uint32_t j = 1; j <= zr; ++j)
                if (wo + j < capw) o[wo + j] = 0ull;
            pos = ok ? pos + len : pos;
            lit = ok ? (isl ? lit - 1u : (f ? c9 : 0u)) : lit;
            wo = ok ? wo + 1u + zr : wo;
            if (eof) {
                st = ST_EOF;
                act = false;
            }
        }
        if (mine && st == ST_OK && wo > capw) st = ST_SPACE;
        // ---- 4. store the OK units' words, flattened by 16-B pairs -----------------------------
        const uint32_t npair = (mine && st == ST_OK) ? (wo + 1) >> 1 : 0u;
        const uint32_t ipr = wave_incl_sum(npair, lane);
        const uint32_t NPR = readlane(ipr, g - 1);
        opf[lane] = mine ? ipr - npair : 0xFFFFFFFFu;
        wave_lds_sync();  // step 3's output words and the pair prefix are visible
        const uint32_t NPR64 = (NPR + kWave - 1) / kWave * kWave;  // wave-uniform trip count
        for (uint32_t j = lane; j < NPR64; j += kWave) {
            const uint32_t jj = j < NPR ? j : (NPR ? NPR - 1 : 0u);
            const uint32_t k = sg_find(opf, g, jj);
            const uint64_t d = (uint64_t)__shfl((long long)dst, (int)k, kWave);
            const uint32_t k0 = (uint32_t)__shfl((int)(ipr - npair), (int)k, kWave);
            const uint32_t kw = (uint32_t)__shfl((int)wo, (int)k, kWave);
            const uint32_t kb = (uint32_t)__shfl((int)wb, (int)k, kWave);
            if (j < NPR) {
                const uint32_t w = 2 * (jj - k0);
                uint64_t* const gd = reinterpret_cast<uint64_t*>(d) + w;
                const uint64_t x0 = pout[kb + w];
                if (w + 1 < kw) {
                    const uint64_t x1 = pout[kb + w + 1];
                    const u32x4 vv = {(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
                    *reinterpret_cast<u32x4*>(gd) = vv;
                } else {
                    *gd = x0;
                }
            }
        }
        if (mine) {
            out_len[unit] = st == ST_OK || st == ST_SPACE ? 8ull * wo : 0ull;
            status[unit] = st;
        }
        cursor += g;
    }
}

// ---------------------------------------------------------------------------
// Message.validate, batched (message.zig:699-969)
// ---------------------------------------------------------------------------
// Lane per framed message. Each lane runs Message.init's segment-table parse
// (message.zig:341-394) and then the reference's recursive depth-first walk
// (validatePointer and the struct / list / far / inline-composite validators) as a
// state machine over an explicit stack of pointer runs:
// - The walk is a chain of dependent reads, and lanes of a wave sit in different
//   states. So every turn of the wave's loop issues at most ONE read per lane (the
//   4/8/16 bytes its walk needs next) and then advances each lane through all the work
//   that needs no memory. No turn serialises several round trips for the wave.
// - A persistent grid: each wave owns a contiguous range of messages and its lanes take
//   the next one as they finish (a wave-uniform cursor, no atomics), so a long message
//   does not idle the other 63 lanes.
// - A frame is one run of pointer words still to visit: the current element's remaining
//   pointers (pleft of pw, from byte `cur` of segment `seg`) and the elements after it
//   (eleft, each dw data words then pw pointers), at the nesting value the reference
//   passes to validatePointer for them. Pushing a frame spends a nesting level, so a lane
//   never holds more than nesting_limit frames. The first kVdLds live in LDS, deeper ones
//   (up to kVdDepth) in the lane's private scratch. A frame keeps its nesting value in 6
//   bits, relative to base = max(nesting_limit - 64, 0): a message that needs a frame
//   below base (only with nesting_limit > 64) is handed, untouched, to a deep list, and the
//   DEEP instance of the kernel validates the listed messages with the frames in global
//   scratch (depth_cap frames per lane, the nesting value in a u32 beside each).
// - Segment offsets: the first kVdSegs segments' byte offsets are kept in LDS from the
//   header parse; one more (the last sought) in registers; any other is sought again by
//   reading the segment table.
// Visiting order, limit consumption and every check follow the reference line by line,
// so a message's status is the first error the reference raises.
constexpr uint32_t kVdDepth = 64;  // frames per lane in LDS + private scratch (the reference default limit)
// Largest nesting limit the device applies (a larger one is clamped to it): 2^18 pointer
// levels, far past the depth at which the reference's recursive validatePointer exhausts
// its thread stack. It bounds the DEEP kernel's frame stack and every far-pointer chain.
constexpr uint32_t kVdMaxNest = 1u << 18;
constexpr uint32_t kVdLds = 8;  // stack frames per lane held in LDS
constexpr uint32_t kVdSegs = 4;          // segments per lane whose offsets are held in LDS

enum : uint32_t {
    VK_IDLE,     // no message: take the next one
    VK_EXIT,     // the wave's range is done
    VK_META,     // read in_off / in_len
    VK_COUNT,    // read the segment count (and segment 0's size)
    VK_SIZES,    // read segment sizes (Message.init's truncation check)
    VK_PTR,      // read a pointer word: validatePointer (also a single far's landing pad)
    VK_LAND2,    // read a double far's 16-B landing pad
    VK_TAG,      // read an inline-composite tag word
    VK_SEEK,     // read segment sizes to find a segment's offset
    VK_REQ_PTR,  // (no read) issue the read of the next pointer word
};

__device__ __forceinline__ uint64_t ld_u64(const uint8_t* p) {  // unaligned-safe 8-B load
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ int64_t ptr_offset_words(uint64_t w) {  // message.zig:11-18
    const uint32_t raw = (uint32_t)((w >> 2) & 0x3FFFFFFFu);
    return (raw & 0x20000000u) ? (int64_t)raw - ((int64_t)1 << 30) : (int64_t)raw;
}

// Deep-path arguments (VdDeep): the list of deferred messages and its count; for the DEEP
// instance also the global frame stack (frame i of global lane g at [i * lanes + g]) with the
// frames' nesting values, its depth and the lanes of the grid that take messages.
struct VdDeep {
    uint32_t* list = nullptr;
    uint32_t* count = nullptr;
    uint4* stk = nullptr;
    uint32_t* nest = nullptr;
    uint32_t depth_cap = 0;
    uint32_t lanes = 0;
};

template <bool DEEP>
// Occupancy: the compiler's choice (129 VGPRs) gives 3 waves/SIMD; pinned at 4 (127 VGPRs, 4
// spilled) the trees leg runs 1.87 instead of 1.95-1.96 ms; at 5 (78 spilled) 3.42 ms (same box,
// scripts/dev/vd_ab.sh against the round-4 source).
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4, 4))) void validate_kernel(const uint8_t* __restrict__ in,
                                                         const uint64_t* __restrict__ in_off,
                                                         const uint64_t* __restrict__ in_len, uint32_t n,
                                                         uint32_t per_wave, uint64_t seg_limit, uint64_t trav_limit,
                                                         uint32_t nest_limit, int32_t* __restrict__ status,
                                                         uint64_t* __restrict__ words, VdDeep dp) {
    __shared__ uint4 stack_all[DEEP ? 1 : kVdLds * kWave];  // frame f < kVdLds of lane l at [f * 64 + l]
    __shared__ uint32_t segp_all[(kVdSegs + 1) * kWave];  // segment i's start (i <= kVdSegs) at [i * 64 + l]
    uint4 deep[DEEP ? 1 : kVdDepth - kVdLds];            // frames kVdLds.. (private scratch)
    const uint32_t lane = lane_id();
    uint4* const stk = stack_all + (DEEP ? 0 : lane);
    uint32_t* const segp = segp_all + lane;
    const uint64_t glane = (uint64_t)blockIdx.x * kWave + lane;
    if (DEEP) {  // the deferred messages, spread over the grid
        n = *dp.count;
        per_wave = (n + gridDim.x - 1) / gridDim.x;
    }
    // nesting values in the frames are relative to base (6 bits; DEEP: absolute, in dp.nest)
    const uint32_t base = nest_limit > kVdDepth ? nest_limit - kVdDepth : 0u;
    const uint64_t first = (uint64_t)blockIdx.x * per_wave;
    const uint64_t last = first + per_wave < n ? first + per_wave : n;
    uint64_t cursor = first;  // wave-uniform

    uint32_t kind = (DEEP && glane >= dp.lanes) ? VK_EXIT : VK_IDLE;
    uint64_t msg = 0;
    const uint8_t* d = in;
    const uint8_t* laddr = in;  // the pending read
    uint32_t lsz = 0;
    uint64_t len = 0, rem = 0;
    uint32_t nseg = 0, si = 0, depth = 0;
    uint64_t acc = 0;
    uint32_t xseg = 0xFFFFFFFFu;  // the sought segment cached in registers
    uint64_t xoff = 0, xlen = 0;
    uint32_t sk_target = 0, sk_i = 0, sk_ret = 0;
    uint64_t sk_acc = 0, sva = 0, svb = 0;
    uint32_t pseg = 0, pnest = 0;  // the pending pointer, or the pending tag's nesting
    uint64_t ppos = 0;
    uint32_t tseg = 0;  // the pending inline-composite tag: segment, position, list word count
    uint64_t tpos = 0, twc = 0;

    const uint64_t glanes = dp.lanes;  // DEEP: the frame stack's lane stride
    auto frame_store = [&](uint32_t i, uint4 f) {
        if (DEEP) dp.stk[(uint64_t)i * glanes + glane] = f;
        else if (i < kVdLds) stk[kWave * i] = f;
        else deep[i - kVdLds] = f;
    };
    auto frame_load = [&](uint32_t i) {
        if (DEEP) return dp.stk[(uint64_t)i * glanes + glane];
        return i < kVdLds ? stk[kWave * i] : deep[i - kVdLds];
    };
    auto frame_nest = [&](uint32_t i, const uint4& f) {
        return DEEP ? dp.nest[(uint64_t)i * glanes + glane] : (f.w >> 26) + base;
    };
    auto finish = [&](int32_t st) {
        status[msg] = st;
        if (words) words[msg] = st == ST_OK ? trav_limit - rem : 0ull;
        kind = VK_IDLE;
    };
    // false: the message was deferred to the deep list (nothing written for it here)
    auto push = [&](uint32_t seg, uint64_t cur, uint32_t pleft, uint32_t pw, uint32_t eleft, uint32_t dw,
                    uint32_t nest) {
        if (DEEP) {
            if (depth >= dp.depth_cap) {  // cannot happen: a frame spends a level and >= 1 word
                finish(ST_NEST);
                return false;
            }
            dp.nest[(uint64_t)depth * glanes + glane] = nest;
        } else if (nest < base) {
            dp.list[atomicAdd(dp.count, 1u)] = (uint32_t)msg;
            kind = VK_IDLE;
            return false;
        }
        frame_store(depth, make_uint4((uint32_t)cur, eleft, pleft | (pw << 16),
                                      dw | (seg << 16) | (DEEP ? 0u : (nest - base) << 26)));
        ++depth;
        return true;
    };
    auto consume = [&](uint64_t w) {  // :710-713
        if (w > rem) return false;
        rem -= w;
        return true;
    };
    auto seg_lookup = [&](uint32_t s, uint64_t& off, uint64_t& slen) {  // s < nseg
        const uint32_t lim = nseg < kVdSegs ? nseg : kVdSegs;
        if (s < lim) {
            off = segp[kWave * s];
            slen = segp[kWave * (s + 1)] - off;
            return true;
        }
        if (s == xseg) {
            off = xoff;
            slen = xlen;
            return true;
        }
        return false;
    };
    auto request = [&](uint32_t k, const uint8_t* a, uint32_t size) {
        kind = k;
        laddr = a;
        lsz = size;
    };
    auto seek_next = [&]() { request(VK_SEEK, d + 4 + 4ull * sk_i, sk_i < sk_target ? 8u : 4u); };
    // find segment s (>= kVdSegs) in the segment table, then re-run state `ret` on (va, vb)
    auto start_seek = [&](uint32_t s, uint32_t ret, uint64_t va, uint64_t vb) {
        sk_target = s;
        sk_i = kVdSegs;
        sk_acc = segp[kWave * kVdSegs];
        sk_ret = ret;
        sva = va;
        svb = vb;
        seek_next();
    };
    auto load_ptr = [&]() {  // read the pointer word at (pseg, ppos)
        uint64_t off, slen;
        if (!seg_lookup(pseg, off, slen)) start_seek(pseg, VK_REQ_PTR, 0, 0);
        else request(VK_PTR, d + off + ppos, 8);
    };
    auto next = [&]() {  // the next pointer of the walk, or the end of the message
        while (depth) {
            uint4 f = frame_load(depth - 1);
            if (f.z & 0xFFFFu) {
                pseg = (f.w >> 16) & 0x3FFu;
                ppos = f.x;
                pnest = frame_nest(depth - 1, f);
                f.x += 8;
                f.z -= 1;
                frame_store(depth - 1, f);
                load_ptr();
                return;
            }
            if (f.y) {
                f.y -= 1;
                f.x += 8 * (f.w & 0xFFFFu);  // the next element's pointer section
                f.z |= f.z >> 16;
                frame_store(depth - 1, f);
                continue;
            }
            --depth;
        }
        finish(ST_OK);
    };
    auto sizes_next = [&]() {  // after segment si - 1: the next sizes, or validate's preamble (:699-708)
        if (si < nseg) {
            request(VK_SIZES, d + 4 + 4ull * si, si + 1 < nseg ? 8u : 4u);
            return;
        }
        if (nseg > seg_limit) return finish(ST_SEGLIMIT);
        if (segp[kWave] - segp[0] < 8) return finish(ST_TRUNC);
        pseg = 0;
        ppos = 0;
        pnest = nest_limit;
        load_ptr();
    };
    auto add_size = [&](uint32_t words_) {  // Message.init :376-383
        acc += 8ull * words_;
        if (acc > len) return false;
        ++si;
        if (si <= kVdSegs) segp[kWave * si] = (uint32_t)acc;
        return true;
    };
    // list content (non-composite) at co of segment s: listContentBytes / bounds / consume (:871-896)
    auto plain_list = [&](uint32_t s, uint64_t co, uint64_t w, uint32_t nest) {
        const uint32_t es = (uint32_t)(w >> 32) & 7u;
        const uint64_t wc = w >> 35;
        const uint64_t bytes = es == 0 ? 0 : es == 1 ? (wc + 7) / 8 : es == 2 ? wc : es == 3 ? 2 * wc
                             : es == 4 ? 4 * wc : 8 * wc;  // listContentBytes (:65-79)
        uint64_t off, slen;
        seg_lookup(s, off, slen);
        if (co > slen || bytes > slen - co) return finish(ST_OOB);
        if (!consume((bytes + 7) / 8)) return finish(ST_TRAV);  // listContentWords (:81-86)
        if (es == 6 && wc && !push(s, co, 1, 1, (uint32_t)(wc - 1), 0, nest)) return;
        next();
    };
    // inline-composite elements from a tag (:940-968 with layout A, :846-868, :911-926)
    auto composite = [&](uint32_t s, uint64_t eo, uint64_t tag, uint64_t total_words, uint32_t nest) {
        const uint64_t count = (uint64_t)ptr_offset_words(tag), dw = (tag >> 32) & 0xFFFFu, pw = tag >> 48;
        uint64_t off, slen;
        seg_lookup(s, off, slen);
        if (eo > slen || total_words * 8 > slen - eo) return finish(ST_OOB);
        if (!consume(total_words)) return finish(ST_TRAV);
        if (pw && count && !push(s, eo + 8 * dw, (uint32_t)pw, (uint32_t)pw, (uint32_t)(count - 1), (uint32_t)dw, nest))
            return;
        next();
    };

    for (;;) {
        // ---- take new messages ---------------------------------------------------------------
        const uint64_t idle = __ballot(kind == VK_IDLE);
        if (idle) {
            if (cursor < last) {
                if (kind == VK_IDLE) {
                    const uint64_t id = cursor + __popcll(idle & ((1ull << lane) - 1));
                    if (id < last) {
                        msg = DEEP ? dp.list[id] : id;
                        kind = VK_META;
                    } else {
                        kind = VK_EXIT;
                    }
                }
                cursor += __popcll(idle);
            } else if (kind == VK_IDLE) {
                kind = VK_EXIT;
            }
        }
        if (__ballot(kind != VK_EXIT) == 0) break;
        // ---- the one read of this turn -----------------------------------------------------------
        uint64_t va = 0, vb = 0;
        if (kind == VK_META) {
            va = in_off[msg];
            vb = in_len[msg];
        } else if (kind >= VK_COUNT && kind <= VK_SEEK) {
            if (lsz == 4) va = ld_u32(laddr);
            else va = ld_u64(laddr);
            if (lsz == 16) vb = ld_u64(laddr + 8);
        }
        // ---- advance the lane to its next read --------------------------------------------------
        for (bool go = true; go;) {
            go = false;
            switch (kind) {
            case VK_META:
                d = in + va;
                len = vb;
                rem = trav_limit;
                depth = 0;
                xseg = 0xFFFFFFFFu;
                if (len >= 0x100000000ull) finish(ST_ARG);  // byte offsets in the frames are u32
                else if (len < 4) finish(ST_EOS);
                else request(VK_COUNT, d, len >= 8 ? 8u : 4u);
                break;
            case VK_COUNT: {  // Message.init :341-371
                const uint32_t m1 = (uint32_t)va;
                if (m1 == 0xFFFFFFFFu) { finish(ST_SEGCOUNT); break; }
                if ((uint64_t)m1 + 1 > kMsgMaxSegs) { finish(ST_SEGLIMIT); break; }
                nseg = m1 + 1;
                acc = 4ull * (1 + nseg + ((nseg & 1) ? 0 : 1));
                if (acc > len) { finish(ST_TRUNC); break; }
                segp[0] = (uint32_t)acc;
                si = 0;
                if (lsz == 8 && !add_size((uint32_t)(va >> 32))) { finish(ST_TRUNC); break; }
                sizes_next();
                break;
            }
            case VK_SIZES:
                if (!add_size((uint32_t)va) || (lsz == 8 && !add_size((uint32_t)(va >> 32)))) {
                    finish(ST_TRUNC);
                    break;
                }
                sizes_next();
                break;
            case VK_SEEK: {
                bool found = false;
                for (uint32_t h = 0; h < lsz / 4 && !found; ++h) {
                    const uint32_t sz = (uint32_t)(va >> (32 * h));
                    if (sk_i == sk_target) {
                        xseg = sk_target;
                        xoff = sk_acc;
                        xlen = 8ull * sz;
                        found = true;
                    } else {
                        sk_acc += 8ull * sz;
                        ++sk_i;
                    }
                }
                if (!found) {
                    seek_next();
                    break;
                }
                kind = sk_ret;  // re-run the state that needed the segment
                va = sva;
                vb = svb;
                go = true;
                break;
            }
            case VK_REQ_PTR:
                load_ptr();
                break;
            case VK_PTR: {  // validatePointer (:715-734) on the word at (pseg, ppos)
                const uint64_t w = va;
                if (w == 0) { next(); break; }
                if (pnest == 0) { finish(ST_NEST); break; }
                if (pseg >= nseg) { finish(ST_SEGID); break; }
                const uint32_t type = (uint32_t)w & 3u;
                if (type == 3) { finish(ST_PTR); break; }
                const uint32_t nest = pnest - 1;
                if (type == 0) {  // validateStructPointer (:774-812)
                    const uint64_t ds = (w >> 32) & 0xFFFFu, pc = w >> 48;
                    const int64_t so_s = (int64_t)ppos + 8 + ptr_offset_words(w) * 8;
                    uint64_t off, slen;
                    seg_lookup(pseg, off, slen);
                    if (so_s < 0 || (uint64_t)so_s > slen || (ds + pc) * 8 > slen - (uint64_t)so_s) {
                        finish(ST_OOB);
                        break;
                    }
                    if (!consume(ds + pc)) { finish(ST_TRAV); break; }
                    if (pc && !push(pseg, (uint64_t)so_s + 8 * ds, (uint32_t)pc, (uint32_t)pc, 0, 0, nest)) break;
                    next();
                    break;
                }
                if (type == 1) {  // validateListPointer (:814-897)
                    const int64_t c = (int64_t)ppos + 8 + ptr_offset_words(w) * 8;
                    if (c < 0) { finish(ST_OOB); break; }
                    if (((w >> 32) & 7u) != 7) { plain_list(pseg, (uint64_t)c, w, nest); break; }
                    // inline composite: resolveInlineCompositeList (:563-609) reads the tag at c
                    uint64_t off, slen;
                    seg_lookup(pseg, off, slen);
                    if ((uint64_t)c + 8 > slen) { finish(ST_OOB); break; }
                    tseg = pseg;
                    tpos = (uint64_t)c;
                    twc = w >> 35;
                    pnest = nest;
                    request(VK_TAG, d + off + tpos, 8);
                    break;
                }
                // validateFarPointer (:736-772) + resolveFarLandingPad (:430-437)
                const bool dbl = (w >> 2) & 1u;
                const uint64_t landing = ((w >> 3) & 0x1FFFFFFFu) * 8;
                const uint32_t fseg = (uint32_t)(w >> 32);
                if (fseg >= nseg) { finish(ST_SEGID); break; }
                uint64_t off, slen;
                if (!seg_lookup(fseg, off, slen)) { start_seek(fseg, VK_PTR, va, vb); break; }
                if (landing + (dbl ? 16 : 8) > slen) { finish(ST_OOB); break; }
                pnest = nest;
                if (!dbl) {  // the landing word is validatePointer'd at the same nesting
                    pseg = fseg;
                    ppos = landing;
                    request(VK_PTR, d + off + landing, 8);
                } else {
                    request(VK_LAND2, d + off + landing, 16);
                }
                break;
            }
            case VK_LAND2: {  // :754-771 (nesting: pnest)
                const uint64_t lw = va, tw = vb;
                if ((lw & 3) != 2 || ((lw >> 2) & 1u)) { finish(ST_FAR); break; }
                const uint32_t s2 = (uint32_t)(lw >> 32);
                if (s2 >= nseg) { finish(ST_SEGID); break; }
                uint64_t off, slen;
                if (!seg_lookup(s2, off, slen)) { start_seek(s2, VK_LAND2, va, vb); break; }
                const uint64_t eo = ((lw >> 3) & 0x1FFFFFFFu) * 8;
                if ((tw & 3) == 0) {  // validateInlineCompositeTag (:929-968), layout A
                    if (ptr_offset_words(tw) < 0) { finish(ST_ICP); break; }
                    const uint64_t tot = (uint64_t)ptr_offset_words(tw) * (((tw >> 32) & 0xFFFFu) + (tw >> 48));
                    composite(s2, eo, tw, tot, pnest);
                    break;
                }
                if ((tw & 3) != 1) { finish(ST_FAR); break; }
                if (((tw >> 32) & 7u) != 7) { plain_list(s2, eo, tw, pnest); break; }
                // layout B (:827-869): the tag is at the landing pad's target
                if (eo + 8 > slen) { finish(ST_OOB); break; }
                tseg = s2;
                tpos = eo;
                twc = tw >> 35;
                request(VK_TAG, d + off + eo, 8);
                break;
            }
            case VK_TAG: {  // the tag checks of :583-600 / :833-851, then the elements
                const uint64_t tag = va;
                if ((tag & 3) != 0 || ptr_offset_words(tag) < 0) { finish(ST_ICP); break; }
                const uint64_t count = (uint64_t)ptr_offset_words(tag);
                if (count * (((tag >> 32) & 0xFFFFu) + (tag >> 48)) > twc) { finish(ST_ICP); break; }
                composite(tseg, tpos + 8, tag, twc, pnest);
                break;
            }
            default:
                break;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Reader.readPackedMessage, batched (reader.zig:84-156)
// ---------------------------------------------------------------------------
// Unit i is one reader's buffered packed stream; one message is decoded from its
// front (launch_read_message):
//   1. read_header_kernel: lane per unit, decodes records until the segment table
//      is complete (one record for a 1-segment message) and writes the framed
//      length to out_len, or the header error to status;
//      (ROUTE: messages of at most kRdWordsMax framed words kStWords, longer ones kStNeedWalk);
//   2. messages of more than kRdWordsMax words: decode_index_kernel<true, kRdWalk> (the walk
//      alone, consumed) and decode_index_kernel<false, kRdGate> (the records over in_len =
//      consumed), then the fill pass and the full-path fallback over in_len = consumed;
//   3. the others: decode_words_kernel<true> (round 6), which stops each lane's walk at the
//      first record boundary that reaches the framed length and applies the reader's
//      overshoot / end-of-stream rules there; consumed = the bytes it walked.
constexpr uint64_t kMaxTotalWords = 8ull * 1024 * 1024;  // reader.zig:6
constexpr uint64_t kMaxSegments = 512;                   // message.zig:310
constexpr uint64_t kHdrMaxWords = 257;                   // (1 + 512 + pad) u32 = 257 words

// Pass 1. Checks follow the reference's order: a record cut short by the end of
// the stream (EndOfStream), then after the first record InvalidSegmentCount /
// SegmentCountLimitExceeded (reader.zig:121-125), then once header_bytes are
// decoded MessageTooLarge (:140). Segment sizes are summed from the header's
// words as the records produce them (zero words add nothing). packed_header returns the
// status and, when OK, the framed length in `needed`.
__device__ int32_t packed_header(const uint8_t* __restrict__ p, uint64_t P, uint64_t& needed) {
    uint64_t r = 0;          // read cursor
    uint64_t words = 0;      // decoded words (out.items.len / 8)
    uint64_t count = 0;      // segment count (set by word 0)
    uint32_t count_m1 = 0;
    uint64_t total = 0;      // sum of the sizes decoded so far
    needed = 0;
    for (;;) {
        if (r >= P) return ST_EOS;  // :95 readByte
        const uint32_t t = p[r++];
        uint64_t w0 = 0;
        uint32_t c = 0;
        const uint8_t* lit = p;
        if (t == 0x00) {  // :96-99
            if (r >= P) return ST_EOS;
            c = p[r++];
        } else if (t == 0xFF) {  // :100-110
            if (P - r < 9) return ST_EOS;
            w0 = gload_u64_unaligned(p + r);
            c = p[r + 8];
            r += 9;
            if (P - r < 8ull * c) return ST_EOS;
            lit = p + r;
            r += 8ull * c;
        } else {  // :111-119
            if (P - r < (uint64_t)__popc(t)) return ST_EOS;
            for (uint32_t k = 0; k < 8; ++k)
                if ((t >> k) & 1u) w0 |= (uint64_t)p[r++] << (8 * k);
        }
        // the record's words that hold header u32s: u32 j of the frame is
        // segment count - 1 (j = 0) or the size of segment j - 1 (1 <= j <= count)
        const uint64_t nw = 1ull + c;
        if (words == 0) {
            count_m1 = (uint32_t)w0;
            count = (uint64_t)count_m1 + 1;
        }
        if (t != 0x00) {
            for (uint64_t i = 0; i < nw && words + i < kHdrMaxWords; ++i) {
                const uint64_t w = i == 0 ? w0 : gload_u64_unaligned(lit + 8 * (i - 1));
                const uint64_t j = 2 * (words + i);
                if (j >= 1 && j <= count) total += (uint32_t)w;
                if (j + 1 <= count) total += w >> 32;
            }
        }
        words += nw;
        // :121-144 (out.items.len >= 4 after any record)
        if (count_m1 == 0xFFFFFFFFu) return ST_SEGCOUNT;
        if (count > kMaxSegments) return ST_SEGLIMIT;
        const uint64_t header_bytes = 4 * (1 + count + ((count & 1) ? 0 : 1));
        if (8 * words >= header_bytes) {
            if (total > kMaxTotalWords) return ST_TOOLARGE;
            needed = header_bytes + 8 * total;
            return ST_OK;
        }
    }
}

// ROUTE (launch_read_message): a message of at most kRdWordsMax framed words goes to the words
// decoder (kStWords), a longer one to the walk passes (kStNeedWalk); errors stand.
template <bool ROUTE>
__global__ __launch_bounds__(kBlock) void read_header_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ in_off,
                                                             const uint64_t* __restrict__ in_len, uint32_t n,
                                                             uint64_t* __restrict__ out_len,
                                                             uint64_t* __restrict__ consumed,
                                                             int32_t* __restrict__ status) {
    const uint32_t unit = blockIdx.x * kBlock + threadIdx.x;
    if (unit >= n) return;
    uint64_t needed = 0;
    const int32_t st = packed_header(in + in_off[unit], in_len[unit], needed);
    status[unit] = (ROUTE && st == ST_OK) ? ((needed >> 3) <= kRdWordsMax ? kStWords : kStNeedWalk) : st;
    out_len[unit] = st == ST_OK ? needed : 0;
    consumed[unit] = 0;
}

// ---------------------------------------------------------------------------
// Resumable framing of packed socket streams (capnp_packed_framer_*).
// Each connection's unconsumed packed bytes stay in a device arena between reads; a read
// appends only its new bytes, and the walk to the message end resumes where the previous
// read left it, so a message split over k reads is uploaded once and walked once
// (framing.zig:42-90 keeps expected_total across pushes; reader.zig:84-156 is one pass).
// ---------------------------------------------------------------------------

// Batched byte copies (dst, src, len as absolute device addresses, 3 u64 per job): a block per
// job (grid-stride); lane t stores destination-aligned 16-B chunks from unaligned 16-B loads
// (gfx950 global loads take any alignment), the two partial edge chunks byte by byte.
// Jobs never overlap (appends from the staging buffer, region moves into fresh regions).
__global__ __launch_bounds__(256) void copy_jobs_kernel(const uint64_t* __restrict__ jobs, uint32_t nj) {
    for (uint32_t j = blockIdx.x; j < nj; j += gridDim.x) {
        uint8_t* const dst = reinterpret_cast<uint8_t*>(jobs[3 * j]);
        const uint8_t* const src = reinterpret_cast<const uint8_t*>(jobs[3 * j + 1]);
        const uint64_t len = jobs[3 * j + 2];
        if (len == 0) continue;
        const uint64_t d0 = reinterpret_cast<uint64_t>(dst), d1 = d0 + len;
        const uint64_t c0 = d0 & ~15ull, c1 = (d1 + 15) & ~15ull;  // 16-B chunks touched
        for (uint64_t c = c0 + 16ull * threadIdx.x; c < c1; c += 16ull * blockDim.x) {
            const uint64_t lo = c < d0 ? d0 : c, hi = c + 16 > d1 ? d1 : c + 16;
            if (lo == c && hi == c + 16) {
                uint4 v;
                __builtin_memcpy(&v, src + (c - d0), 16);
                *reinterpret_cast<uint4*>(c) = v;
            } else {
                for (uint64_t b = lo; b < hi; ++b) *reinterpret_cast<uint8_t*>(b) = src[b - d0];
            }
        }
    }
}

// The walk of a connection's held bytes, message after message: a wave per
// listed connection. Each message's framed length comes from its header (packed_header on lane
// 0; need[c] already holds it when the previous read decoded the header), then the walk to its
// end goes window by window (wv_stage / wv_resolve: 4.6-KB windows resolved in parallel),
// counting the words of complete records only, from packed byte X of the message, where the
// previous read left it. A message ends at the first record after which the words reach
// need / 8 (reader.zig:90-93 and 146-153: OK with the packed bytes up to that record's end, or
// InvalidPackedMessage when the record produced more); its packed length and framed length go
// to tab[2 (i M + m)] / [+ 1] and the next message starts there. The walk stops after M
// messages (status OK: the host walks again), at an error, or at the held bytes' end
// (EndOfStream): need / X / W then describe the current message for the next read (X from
// its start; need 0 while its header is incomplete) and cnt[i] the messages found. A message
// found whole that the caller's frames buffer could not take comes back with W = need / 8 and
// X at its end: the next walk takes it as found without walking it again.
// base / avail: the connection's first held byte in the arena and the bytes it holds.
__global__ __launch_bounds__(kWvBlock) void frame_walk_kernel(const uint8_t* __restrict__ arena,
                                                              const uint32_t* __restrict__ list, uint32_t nl,
                                                              const uint64_t* __restrict__ base,
                                                              const uint64_t* __restrict__ avail,
                                                              uint64_t* __restrict__ need,
                                                              uint64_t* __restrict__ Xs, uint64_t* __restrict__ Ws,
                                                              int32_t* __restrict__ status,
                                                              const WinEnt* __restrict__ spec,
                                                              const uint32_t* __restrict__ spec_first, uint32_t M,
                                                              uint32_t* __restrict__ cnt, uint32_t* __restrict__ tab) {
    __shared__ __attribute__((aligned(16))) uint8_t pk_all[kWvWaves * kWvPk];
    __shared__ __attribute__((aligned(16))) uint8_t mk_all[kWvWaves * kWvWin];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* const pk = pk_all + wave * kWvPk;
    uint8_t* const mk = mk_all + wave * kWvWin;
    for (uint32_t i = blockIdx.x * kWvWaves + wave; i < nl; i += gridDim.x * kWvWaves) {
        const uint32_t c = __builtin_amdgcn_readfirstlane(list[i]);
        const uint8_t* const src = arena + base[c];
        const uint64_t P = avail[c];
        uint64_t L = need[c];   // the current message's framed bytes (0: header not decoded)
        uint64_t m0 = 0;        // its first packed byte
        uint64_t x = Xs[c], wd = Ws[c];
        uint32_t nm = 0;
        int32_t st = ST_EOS;
        // windows at fixed positions x0 + j * kWvWin; with a spec table (window_spec_kernel over
        // [x0, P), computed for all windows at once), a window the message neither ends in nor
        // runs out of bytes in is crossed by a table lookup: its exit and word count from the
        // entry d the chain arrives at
        const uint64_t x0 = x;
        const uint32_t sf = spec_first ? __builtin_amdgcn_readfirstlane(spec_first[i]) : kWinNone;
        for (;;) {
            if (L == 0) {  // the next message's header (x == m0, wd == 0)
                if (nm == M) {
                    st = ST_OK;
                    break;
                }
                uint64_t nd = 0;
                int32_t hs = ST_EOS;
                if (lane == 0) hs = packed_header(src + m0, P - m0, nd);
                hs = (int32_t)readlane((uint32_t)hs, 0);
                if (hs != ST_OK) {
                    st = hs;
                    break;
                }
                L = ((uint64_t)readlane((uint32_t)(nd >> 32), 0) << 32) | readlane((uint32_t)nd, 0);
            }
            const uint64_t Lw = L >> 3;  // framed words (L is a multiple of 8)
            bool ended = wd >= Lw;       // walked whole by an earlier pass (X at its end)
            while (!ended && x < P) {
                const uint64_t j = (x - x0) / kWvWin;
                const uint64_t Xj = x0 + j * kWvWin;
                const uint32_t d = (uint32_t)(x - Xj);
                if (sf != kWinNone) {
                    const WinEnt* const e = spec + sf + j;
                    const uint64_t vm = e->valid;
                    if (d < kWinD && ((vm >> d) & 1)) {
                        const int32_t dl = e->delta[d];
                        const uint32_t ex = e->exit;
                        if (dl != kDeltaEof && ex != kEOFX) {
                            const uint64_t words = (uint64_t)((int64_t)e->total + dl);
                            if (wd + words < Lw) {
                                wd += words;
                                x = Xj + ex;
                                continue;
                            }
                        }
                    }
                }
                // the window walked exactly from entry d: the message ends in it, the held bytes
                // end in it, or the table does not know entry d
                const WvWin w = wv_stage(pk, mk, src, P, Xj, lane);
                uint32_t ent, cs, ce;
                const uint32_t xw = wv_resolve(pk, mk, w, d, lane, ent, cs, ce);
                // the lane's complete records (a record past the held bytes ends the chain)
                uint32_t words = 0, stop = kEOFX;
                for (uint32_t r = ent; r < ce;) {
                    uint32_t t = pk[w.sh + r];
                    uint32_t b1 = pk[w.sh + r + 1];
                    uint32_t c9 = pk[w.sh + r + 9];
                    asm volatile("" : "+v"(t), "+v"(b1), "+v"(c9));
                    const uint32_t len = wv_len(t, c9);
                    if ((uint64_t)r + len > w.rem) {
                        stop = r;
                        break;
                    }
                    words += 1u + ((t == 0u) ? b1 : 0u) + ((t == 0xFFu) ? c9 : 0u);
                    r += len;
                }
                const uint32_t incl = wave_incl_sum(words, lane);
                const uint32_t total = readlane(incl, kWave - 1);
                if (wd + total >= Lw) {  // the message ends in this window
                    const uint64_t bm = __ballot(wd + incl >= Lw);
                    const uint32_t f = (uint32_t)__builtin_ctzll(bm);
                    uint32_t end = 0, over = 0;
                    if (lane == f) {
                        uint64_t acc = wd + incl - words;
                        for (uint32_t r = ent;;) {
                            const uint32_t t = pk[w.sh + r], b1 = pk[w.sh + r + 1], c9 = pk[w.sh + r + 9];
                            acc += 1u + ((t == 0u) ? b1 : 0u) + ((t == 0xFFu) ? c9 : 0u);
                            r += wv_len(t, c9);
                            if (acc >= Lw) {
                                end = r;
                                over = acc != Lw;
                                break;
                            }
                        }
                    }
                    end = readlane(end, f);
                    over = readlane(over, f);
                    if (over) {
                        st = ST_OVERSHOOT;
                    } else {
                        x = Xj + end;
                        ended = true;
                    }
                    break;
                }
                if (xw == kEOFX) {  // the chain stops at a record the bytes do not hold yet
                    const uint64_t bm = __ballot(stop != kEOFX);
                    x = bm ? Xj + readlane(stop, (uint32_t)__builtin_ctzll(bm)) : x;
                    wd += total;
                    break;
                }
                x = Xj + xw;
                wd += total;
            }
            if (!ended) break;  // EndOfStream (x / wd saved) or the overshoot
            if (lane == 0) {
                tab[2 * ((uint64_t)i * M + nm)] = (uint32_t)(x - m0);
                tab[2 * ((uint64_t)i * M + nm) + 1] = (uint32_t)L;
            }
            ++nm;
            m0 = x;
            wd = 0;
            L = 0;
        }
        if (lane == 0) {
            need[c] = st == ST_EOS ? L : 0;
            Xs[c] = st == ST_EOS ? x - m0 : 0;
            Ws[c] = st == ST_EOS ? wd : 0;
            status[c] = st;
            cnt[i] = nm;
        }
    }
}

// ---------------------------------------------------------------------------
// synthetic generator and offset scan
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t seed, uint64_t unit, uint64_t word) {
    uint64_t x = seed ^ (unit * 0x9E3779B97F4A7C15ULL) ^ (word * 0xC2B2AE3D27D4EB4FULL);
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ void generate_kernel(uint8_t* __restrict__ out, uint64_t n_units, uint64_t words_per_unit,
                                uint64_t unit_base, uint64_t seed, uint32_t thr) {
    const uint64_t total = n_units * words_per_unit;
    for (uint64_t gw = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; gw < total;
         gw += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t u = gw / words_per_unit, w = gw - u * words_per_unit;
        uint64_t h = mix64(seed, unit_base + u, w);
        uint64_t h2 = mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL, unit_base + u, w);
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t r = (uint32_t)(h >> (8 * k)) & 0xFF;
            uint32_t x = (uint32_t)(h2 >> (8 * k)) & 0xFF;
            uint64_t b = (r < thr) ? 0 : (1 + x % 255);
            v |= b << (8 * k);
        }
        *reinterpret_cast<uint64_t*>(out + 8 * gw) = v;
    }
}

constexpr int kScanItems = 8;
constexpr int kScanTile = 256 * kScanItems;

// block-local exclusive scan of u64 lengths; writes the block total to partial[blockIdx.x]
__global__ __launch_bounds__(256) void scan_local_kernel(const uint64_t* __restrict__ len, uint32_t n,
                                                         uint64_t* __restrict__ off,
                                                         uint64_t* __restrict__ partial) {
    __shared__ uint64_t wsum[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + tid * kScanItems;
    uint64_t v[kScanItems];
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = (base + k < n) ? len[base + k] : 0;
        t += v[k];
    }
    uint64_t x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t pre = 0;
    for (uint32_t q = 0; q < wave; ++q) pre += wsum[q];
    uint64_t run = pre + x - t;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) off[base + k] = run;
        run += v[k];
    }
    if (tid == 255) partial[blockIdx.x] = pre + x;
}

// single-block exclusive scan of the partials (in place), then base added
__global__ __launch_bounds__(1024) void scan_partials_kernel(uint64_t* __restrict__ partial, uint32_t np,
                                                             uint64_t base, uint64_t* __restrict__ off_last,
                                                             uint32_t n) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) carry_s = base;
    __syncthreads();
    for (uint32_t b = 0; b < np; b += 1024) {
        uint64_t v = (b + tid < np) ? partial[b + tid] : 0;
        uint64_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint64_t y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint64_t pre = carry_s;
        for (uint32_t q = 0; q < wave; ++q) pre += wsum[q];
        if (b + tid < np) partial[b + tid] = pre + x - v;
        __syncthreads();
        if (tid == 1023) carry_s = pre + x;
        __syncthreads();
    }
    if (tid == 0) off_last[n] = carry_s;
}

__global__ __launch_bounds__(256) void scan_apply_kernel(uint64_t* __restrict__ off, uint32_t n,
                                                         const uint64_t* __restrict__ partial) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    const uint64_t add = partial[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < n) off[base + k] += add;
}

}  // namespace cpk

// ---------------------------------------------------------------------------
// launchers (kernels.h)
// ---------------------------------------------------------------------------
namespace cpk {

static inline uint32_t blocks_for(uint32_t n) { return (n + kWavesPerBlock - 1) / kWavesPerBlock; }

// Grid of the long-list kernels (long_tiles_kernel, long_windows_kernel): at most 64 blocks
// striding over the long list, so they start beside a persistent small-unit grid (a block per
// 256 units of the batch waited ~0.2 ms for slots on config C5, delaying the long-unit chain).
static inline uint32_t list_blocks(uint32_t n) { return std::min((n + 255u) / 256u, 64u); }

// Side stream for the long-unit kernels (encode_tiled_kernel, the decode fallback).
// They select their units by a test on the unit's own lengths, so they need nothing
// from the main kernels and run beside them: a batch whose few long units would
// otherwise run alone after the main grid (config C5's tail) overlaps them with it.
// fork(): the side stream waits for everything already on the caller's stream;
// join(): the caller's stream waits for the side stream's kernels.
//
// Every (device, caller stream) pair has its own context: side stream, fork/join
// events and long-unit queue, so batches on independent caller streams never wait
// on each other, and a graph captured from one stream shares nothing with eager
// work on another. The context's mutex keeps one caller's record/wait pairs and
// queue reset together. A queue that has to grow is replaced by one of at least twice its
// size (so a stream sees O(log n) replacements): the old one is freed after the stream
// drains, unless a hipGraph capture used it (a captured graph may still reference it; it is
// then kept until capnp_packed_stream_release). Growing is refused during a capture.
// Callers that pass their own workspace (capnp_packed_*_batch_ws) use it as the
// queue instead, so nothing of the library's is baked into their graphs.
struct StreamCtx {
    std::mutex mu;
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    hipStream_t s2 = nullptr;  // a second side stream (CAPNP_PACKED_LAUNCH_MID_SIDE_STREAM: C5's mid units)
    hipEvent_t join2 = nullptr;
    uint32_t* q = nullptr;  // class workspace (queue_bytes): kQHead counters, lists, tile / window table
    uint64_t qcap = 0;
    bool q_captured = false;         // q was used inside a hipGraph capture
    std::vector<uint32_t*> retired;  // replaced queues a capture used (graphs may reference them)
    ~StreamCtx() {
        for (uint32_t* r : retired) (void)hipFree(r);
        if (q) (void)hipFree(q);
        if (s) (void)hipStreamDestroy(s);
        if (s2) (void)hipStreamDestroy(s2);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        if (join2) (void)hipEventDestroy(join2);
    }
};
static std::mutex g_ctx_mu;
// shared_ptr: a batch being enqueued keeps its context alive even if capnp_packed_stream_release
// drops it from the map meanwhile (no use-after-free, whatever the callers do).
static std::map<std::pair<int, uintptr_t>, std::shared_ptr<StreamCtx>> g_ctx;

// Byte offset of the piece-record region (decode: kRecStride per mid-list entry) in the
// class workspace, after the lists and the tile / window table.
static uint64_t rec_region_off(uint32_t n) {
    // lists, serial list, then the tile table (encode) or the window table (decode)
    const uint64_t tiles = tile_tab_off(n) * sizeof(uint32_t) + 16 * ((uint64_t)n + kTileExtra);
    const uint64_t wins = win_tab_off(n) * sizeof(uint32_t) + sizeof(WinEnt) * win_cap(n);
    return ((tiles > wins ? tiles : wins) + 255) & ~255ull;
}

size_t queue_bytes(uint32_t n) { return rec_region_off(n) + (uint64_t)kRecStride * n; }

// Resident blocks of a kernel across the device (hipOccupancy...), for persistent grids.
template <typename K>
static uint32_t resident_blocks(K kernel, int block, uint32_t fallback_per_cu) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess || per <= 0)
        per = (int)fallback_per_cu;
    return (uint32_t)(cus * per);
}

static bool class_scan_launched();  // CAPNP_PACKED_LAUNCH_CLASS_SCAN (below)

// Class the batch's units (class_count / class_scan / class_scatter) on the caller's stream.
template <int KIND>
static void launch_classes(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                           uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint32_t* q,
                           int32_t* status, hipStream_t stream, uint32_t words_min = ~0u) {
    const uint32_t nb = (n + kClassBlock - 1) / kClassBlock;
    // up to kClassBlock class blocks (1M units), the scatter does the scan itself
    const uint32_t fused = nb >= 1 && nb <= kClassBlock && !class_scan_launched() ? 1u : 0u;
    class_count_kernel<KIND><<<nb, kClassBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, q, status);
    if (!fused) class_scan_kernel<<<1, 1024, 0, stream>>>(q, n, nb, words_min);
    class_scatter_kernel<KIND><<<nb, kClassBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, q, fused,
                                                               words_min);
}

// Launch policy (capnp_packed_set_launch_flags, process-wide; no result depends on it):
//   CAPNP_PACKED_LAUNCH_LONG_INLINE      the long-unit kernels run after the main grid on the
//                                        caller's stream instead of on a side stream;
//   CAPNP_PACKED_LAUNCH_MID_SIDE_STREAM  decode: a batch's mid units on a second side stream,
//                                        launched before the small units' kernel, whose grid then
//                                        takes 85% of its resident size. Round 3:
//                                        C5 decode 0.678 -> 0.660 ms, but the headline (all mid
//                                        units) 2.474 -> 2.499 ms from the extra fork and join.
//   CAPNP_PACKED_LAUNCH_CLASS_SCAN       the class pass's scan as its own kernel (class_scan_kernel)
//                                        also for batches of at most 1M units, whose scatter
//                                        otherwise does it (the path larger batches always take).
static std::atomic<uint32_t> g_launch_flags{0};
uint32_t set_launch_flags(uint32_t f) { return g_launch_flags.exchange(f); }
static bool mid_side_stream() { return g_launch_flags.load(std::memory_order_relaxed) & CAPNP_PACKED_LAUNCH_MID_SIDE_STREAM; }
static bool class_scan_launched() { return g_launch_flags.load(std::memory_order_relaxed) & CAPNP_PACKED_LAUNCH_CLASS_SCAN; }

class SideLaunch {
  public:
    SideLaunch(hipStream_t main, void* ws, size_t ws_bytes) : main_(main), ws_(ws), ws_bytes_(ws_bytes) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return;
        {
            std::lock_guard<std::mutex> g(g_ctx_mu);
            std::shared_ptr<StreamCtx>& c = g_ctx[{dev, reinterpret_cast<uintptr_t>(main)}];
            if (!c) c = std::make_shared<StreamCtx>();
            ctx_ = c;
        }
        lock_ = std::unique_lock<std::mutex>(ctx_->mu);
        if (g_launch_flags.load(std::memory_order_relaxed) & CAPNP_PACKED_LAUNCH_LONG_INLINE) {
            side_ = main_;
            ok_ = true;
            return;
        }
        if (!ctx_->s) {
            if (hipStreamCreateWithFlags(&ctx_->s, hipStreamNonBlocking) != hipSuccess) {
                ctx_->s = nullptr;
                return;
            }
            if (hipEventCreateWithFlags(&ctx_->fork, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ctx_->join, hipEventDisableTiming) != hipSuccess) {
                (void)hipStreamDestroy(ctx_->s);
                ctx_->s = nullptr;
                return;
            }
        }
        side_ = ctx_->s;
        ok_ = true;
    }
    // the stream the long-unit kernels go on (after fork())
    hipStream_t stream() const { return side_; }
    // The side stream waits for everything enqueued on the caller's stream so far.
    hipError_t fork() {
        if (!ok_ || side_ == main_ || forked_) return ok_ ? hipSuccess : hipErrorNotReady;
        hipError_t e = hipEventRecord(ctx_->fork, main_);
        if (e == hipSuccess) e = hipStreamWaitEvent(side_, ctx_->fork, 0);
        if (e == hipSuccess) forked_ = true;
        return e;
    }
    // The class workspace for a batch of n units (queue_bytes); launch_classes must run on it
    // next (class_scan_kernel clears its counters); nullptr when the side stream or the queue
    // cannot be set up.
    uint32_t* queue(uint32_t n) {
        if (!ok_) return nullptr;
        uint32_t* q = nullptr;
        if (ws_) {
            if (ws_bytes_ < queue_bytes(n)) return nullptr;
            q = static_cast<uint32_t*>(ws_);
        } else {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(main_, &cs) != hipSuccess) return nullptr;
            const bool capturing = cs != hipStreamCaptureStatusNone;
            if (ctx_->qcap < n) {
                if (capturing) return nullptr;
                uint64_t cap = 2 * ctx_->qcap;
                cap = cap < n ? n : cap > 0xFFFFFFFFull ? 0xFFFFFFFFull : cap;
                uint32_t* nq = nullptr;
                if (hipMalloc(reinterpret_cast<void**>(&nq), queue_bytes((uint32_t)cap)) != hipSuccess) return nullptr;
                if (ctx_->q) {
                    if (ctx_->q_captured) {
                        ctx_->retired.push_back(ctx_->q);
                    } else {  // only this stream's batches used it (the side stream joins back)
                        if (hipStreamSynchronize(main_) != hipSuccess) {
                            (void)hipFree(nq);
                            return nullptr;
                        }
                        (void)hipFree(ctx_->q);
                    }
                }
                ctx_->q = nq;
                ctx_->qcap = cap;
                ctx_->q_captured = false;
            }
            ctx_->q_captured |= capturing;
            q = ctx_->q;
        }
        return q;  // its head (counters, cursors) is cleared by class_scan_kernel
    }
    // A second side stream, forked like the first (after fork()); the caller's stream when it
    // cannot be set up.
    hipStream_t stream2() {
        if (!forked_) return main_;
        if (forked2_) return ctx_->s2;
        if (!ctx_->s2) {
            if (hipStreamCreateWithFlags(&ctx_->s2, hipStreamNonBlocking) != hipSuccess) {
                ctx_->s2 = nullptr;
                return main_;
            }
            if (hipEventCreateWithFlags(&ctx_->join2, hipEventDisableTiming) != hipSuccess) {
                (void)hipStreamDestroy(ctx_->s2);
                ctx_->s2 = nullptr;
                return main_;
            }
        }
        if (hipStreamWaitEvent(ctx_->s2, ctx_->fork, 0) != hipSuccess) return main_;
        forked2_ = true;
        return ctx_->s2;
    }
    hipError_t join() {
        if (!forked_) return hipSuccess;
        forked_ = false;
        hipError_t e = hipEventRecord(ctx_->join, side_);
        if (e == hipSuccess) e = hipStreamWaitEvent(main_, ctx_->join, 0);
        if (forked2_) {
            forked2_ = false;
            hipError_t e2 = hipEventRecord(ctx_->join2, ctx_->s2);
            if (e2 == hipSuccess) e2 = hipStreamWaitEvent(main_, ctx_->join2, 0);
            if (e == hipSuccess) e = e2;
        }
        return e;
    }
    ~SideLaunch() { (void)join(); }

  private:
    hipStream_t main_;
    void* ws_;
    size_t ws_bytes_;
    std::shared_ptr<StreamCtx> ctx_;  // held until after the join and the unlock
    std::unique_lock<std::mutex> lock_;
    hipStream_t side_ = nullptr;
    bool ok_ = false, forked_ = false, forked2_ = false;
};

// Drop the library's context of a caller stream (its side stream, events and queues, also
// those captured graphs used): after the stream's work is done and before it is destroyed.
hipError_t release_stream(hipStream_t stream, int dev) {
    hipError_t e = hipSuccess;
    if (dev < 0) e = hipGetDevice(&dev);  // contexts are keyed by (device, stream)
    if (e != hipSuccess) return e;
    std::shared_ptr<StreamCtx> c;
    {
        std::lock_guard<std::mutex> g(g_ctx_mu);
        auto it = g_ctx.find({dev, reinterpret_cast<uintptr_t>(stream)});
        if (it == g_ctx.end()) return hipSuccess;
        c = std::move(it->second);
        g_ctx.erase(it);
    }
    std::lock_guard<std::mutex> g(c->mu);  // no batch of this stream is being enqueued
    e = hipStreamSynchronize(stream);
    if (e == hipSuccess && c->s) e = hipStreamSynchronize(c->s);
    return e;  // ~StreamCtx frees the rest
}

// The per-stream queue the library holds for `stream`: its bytes, and how many replaced
// queues it keeps because a capture used them (tests: growth stays bounded).
void stream_queue_info(hipStream_t stream, size_t* bytes, uint32_t* kept) {
    *bytes = 0;
    *kept = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> g(g_ctx_mu);
    auto it = g_ctx.find({dev, reinterpret_cast<uintptr_t>(stream)});
    if (it == g_ctx.end()) return;
    std::lock_guard<std::mutex> g2(it->second->mu);
    *bytes = it->second->q ? queue_bytes((uint32_t)it->second->qcap) : 0;
    *kept = (uint32_t)it->second->retired.size();
}

uint32_t stream_context_count() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> g(g_ctx_mu);
    uint32_t k = 0;
    for (const auto& kv : g_ctx) k += kv.first.first == dev;
    return k;
}

hipError_t launch_encode(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                         int32_t* status, bool write, void* ws, size_t ws_bytes, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // classes (caller's stream), then the long units on the side stream (encode_tiled_kernel
    // over a grid taking units from the queue) beside the small units (a lane each) and the
    // mid units (a wave each) on the caller's stream
    // long-unit workers: up to one wave per unit, at most the resident grid (a batch of a
    // few long units must not get a grid sized by its unit count / 256)
    static const uint32_t tiled_res = resident_blocks(encode_tiled_kernel<true>, kBlock, 3);
    const uint32_t tiled_blocks = min((n + kWavesPerBlock - 1) / kWavesPerBlock, tiled_res);
    const uint32_t mid_blocks = blocks_for(n);  // waves past the mid count return at once
    SideLaunch side(stream, ws, ws_bytes);
    uint32_t* const q = side.queue(n);
    if (!q) return ws ? hipErrorInvalidValue : hipErrorOutOfMemory;
    launch_classes<4>(in, in_off, in_len, n, out, out_off, out_cap, q, status, stream);
    const uint32_t* const mid_count = q + 12;  // bin 0: the units before bin 1
    const uint32_t es_blocks = (n + kEsWaves * kWave - 1) / (kEsWaves * kWave);  // waves past the count exit
    hipError_t e = side.fork();
    if (e != hipSuccess) return e;
    const hipStream_t ss = side.stream();
    const uint32_t* const mid = q + kQHead + 2ull * n;
    static const uint32_t tiles_res = resident_blocks(tile_encode_kernel<kTilesWrite, true>, kBlock, 4);
    // mid units on a second side stream beside the small-unit kernel (LAUNCH_MID_SIDE_STREAM)
    const hipStream_t ms = mid_side_stream() ? side.stream2() : stream;
    long_tiles_kernel<<<list_blocks(n), 256, 0, ss>>>(in_len, n, q);
    if (write) {
        tile_encode_kernel<kTilesSize, true><<<tiles_res, kBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off,
                                                                             out_cap, out_len, status, q);
        tile_encode_kernel<kTilesWrite, true><<<tiles_res, kBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off,
                                                                              out_cap, out_len, status, q);
        encode_tiled_kernel<true><<<tiled_blocks, kBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                    out_len, status, q);
        if (ms != stream)  // LAUNCH_MID_SIDE_STREAM: the mid units beside the small ones
            encode_kernel<true><<<mid_blocks, kBlock, 0, ms>>>(in, in_off, in_len, n, out, out_off, out_cap, out_len,
                                                                status, mid, mid_count);
        encode_stream_kernel<true><<<es_blocks, kEsWaves * kWave, 0, stream>>>(in, in_off, in_len, n, out, out_off,
                                                                               out_cap, out_len, status, q);
        if (ms == stream)
            encode_kernel<true><<<mid_blocks, kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                    out_len, status, mid, mid_count);
    } else {
        tile_encode_kernel<kTilesSize, false><<<tiles_res, kBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off,
                                                                              out_cap, out_len, status, q);
        tile_encode_kernel<kTilesWrite, false><<<tiles_res, kBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off,
                                                                               out_cap, out_len, status, q);
        encode_tiled_kernel<false><<<tiled_blocks, kBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                     out_len, status, q);
        if (ms != stream)
            encode_kernel<false><<<mid_blocks, kBlock, 0, ms>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                 out_len, status, mid, mid_count);
        encode_stream_kernel<false><<<es_blocks, kEsWaves * kWave, 0, stream>>>(in, in_off, in_len, n, out, out_off,
                                                                                out_cap, out_len, status, q);
        if (ms == stream)
            encode_kernel<false><<<mid_blocks, kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                     out_len, status, mid, mid_count);
    }
    e = hipGetLastError();
    const hipError_t j = side.join();
    return e != hipSuccess ? e : j;
}

// Persistent grid of the fill pass: as many blocks as are resident at once
// (hipOccupancy..., LDS/VGPR-bound), each wave striding over the batch with one
// unit in flight ahead.
static uint32_t fill_blocks(uint32_t n) {
    static const uint32_t resident = [] {  // thread-safe one-time init (C++11 static)
        int dev = 0, cus = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, decode_fill_kernel, kFlWaves * kWave, 0) !=
                hipSuccess || per <= 0)
            per = 4;
        return (uint32_t)(cus * per);
    }();
    const uint32_t full = (n + kFlWaves - 1) / kFlWaves;
    return full < resident ? full : resident;
}

// Pass 1 of the indexed decoder: one wave (64 units) per block.
template <bool SIZE_ONLY>
static void launch_index(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n, uint8_t* out,
                         const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                         hipStream_t stream) {
    decode_index_kernel<SIZE_ONLY><<<ix_blocks_for(n), kWave * kIxBw, 0, stream>>>(in, in_off, in_len, n, out, out_off,
                                                                                   out_cap, out_len, status, nullptr);
}

// Grid of the fallback pass for units a first pass declined: it strides over the
// batch reading statuses, so it stays cheap when (as usual) there are none.
static uint32_t fallback_blocks(uint32_t n) {
    const uint32_t full = (n + kWvWaves * kWave - 1) / (kWvWaves * kWave);
    return full < 2048u ? full : 2048u;
}

// Mid-unit decoder (capnp_packed_set_decoder).
static std::atomic<int> g_decoder{CAPNP_PACKED_DECODER_AUTO};
// Small-unit decoder (capnp_packed_set_all_or_nothing): 1 the lane-streaming kernel (default: a
// failed small unit may keep a prefix), 0 the group-staged kernel (all-or-nothing for small units
// too, slower).
static std::atomic<int> g_small{1};
static int small_variant() { return g_small.load(std::memory_order_relaxed); }
int set_all_or_nothing(int on) { return g_small.exchange(on ? 0 : 1) == 0 ? 1 : 0; }
static int decoder_variant() { return g_decoder.load(std::memory_order_relaxed); }
int set_decoder(int v) { return g_decoder.exchange(v); }
bool decoder_built(int v) {
    return v == CAPNP_PACKED_DECODER_AUTO || v == CAPNP_PACKED_DECODER_TWO_PASS || v == CAPNP_PACKED_DECODER_WORDS;
}

hipError_t launch_decode(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                         int32_t* status, bool write, void* ws, size_t ws_bytes, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (!write) {  // size pass (estimateUnpackedSize, message.zig:152-191)
        // Units of at most kFlPieces pieces: the size-only index walk (a lane per unit). Longer
        // units: window-parallel on the side stream (long_windows / window_spec /
        // window_resolve, which yield out_len without any output), those the window table
        // cannot hold by the size-only walk too; units of 2 GiB or more (the walk declines
        // them) by the lane walk after the join.
        SideLaunch side(stream, ws, ws_bytes);
        uint32_t* const q = side.queue(n);
        if (!q) return ws ? hipErrorInvalidValue : hipErrorOutOfMemory;
        launch_classes<2>(in, in_off, in_len, n, nullptr, nullptr, nullptr, q, status, stream);
        hipError_t e = side.fork();
        if (e != hipSuccess) return e;
        static const uint32_t spec_res = resident_blocks(window_spec_kernel, kWvBlock, 4);
        static const uint32_t res_res = resident_blocks(window_resolve_kernel, kWvBlock, 2);
        const uint64_t wcap = win_cap(n);
        const uint32_t win_blocks = (uint32_t)std::min<uint64_t>((wcap + kWvWaves - 1) / kWvWaves, spec_res);
        const uint32_t res_blocks = std::min((n + kWvWaves - 1) / kWvWaves, res_res);
        const hipStream_t ss = side.stream();
        long_windows_kernel<<<list_blocks(n), 256, 0, ss>>>(in_len, n, q);
        window_spec_kernel<<<win_blocks, kWvBlock, 0, ss>>>(in, in_off, in_len, n, q);
        window_resolve_kernel<<<res_blocks, kWvBlock, 0, ss>>>(in, in_off, in_len, n, nullptr, out_len, status, q);
        decode_index_kernel<true><<<ix_blocks_for(n), kWave * kIxBw, 0, ss>>>(in, in_off, in_len, n, nullptr, nullptr, nullptr,
                                                               out_len, status, nullptr, q + serial_off(n), q + 5);
        decode_index_kernel<true><<<ix_blocks_for(n), kWave * kIxBw, 0, stream>>>(in, in_off, in_len, n, nullptr, nullptr, nullptr,
                                                                   out_len, status, nullptr, q + kQHead + 2ull * n,
                                                                   q + 4);
        e = hipGetLastError();
        const hipError_t j = side.join();
        if (e == hipSuccess) e = j;
        if (e != hipSuccess) return e;
        decode_lane_kernel<false, true><<<(n + kBlock - 1) / kBlock, kBlock, 0, stream>>>(
            in, in_off, in_len, n, out, out_off, out_cap, out_len, status);
        return hipGetLastError();
    }
    // index pass, fill pass; the fallback owns the long units from the start
    // (decode_long_unit): it goes first, on the side stream, beside passes 1 and 2
    static const uint32_t sm_res = resident_blocks(decode_small_kernel, kSmBlock, 8);
    const bool mid_stream = mid_side_stream();
    const double sm_frac = mid_stream ? 0.85 : 1.0;  // share of the resident grid
    const uint32_t sm_cap = std::max(1u, (uint32_t)(sm_res * sm_frac));
    const uint32_t sm_blocks = min((n + kSmBlock - 1) / kSmBlock, sm_cap);
    // mid units: the words decoder where it pays (AUTO: class_scan_kernel's rule, from a grid of
    // its resident units) or for all of them (WORDS); the rest two-pass. The words decoder may
    // leave a failed unit's prefix, so all-or-nothing decodes take the two-pass decoder only.
    const bool words = (decoder_variant() == CAPNP_PACKED_DECODER_AUTO ||
                        decoder_variant() == CAPNP_PACKED_DECODER_WORDS) && small_variant() != 0;
    static const uint32_t words_min = resident_blocks(decode_words_kernel<false>, kLwWaves * kWave, 6) * kLwWaves * kWave;
    SideLaunch side(stream, ws, ws_bytes);
    uint32_t* const q = side.queue(n);
    if (!q) return ws ? hipErrorInvalidValue : hipErrorOutOfMemory;
    launch_classes<1>(in, in_off, in_len, n, out, out_off, out_cap, q, status, stream,
                      !words ? ~0u : (decoder_variant() == CAPNP_PACKED_DECODER_WORDS ? 0u : words_min));
    hipError_t e = side.fork();
    if (e != hipSuccess) return e;
    // long units, window-parallel (window table) or, if the table is full, serial
    static const uint32_t long_res = resident_blocks(decode_wave_kernel<kWvLong>, kWvBlock, 4);
    static const uint32_t spec_res = resident_blocks(window_spec_kernel, kWvBlock, 4);
    static const uint32_t res_res = resident_blocks(window_resolve_kernel, kWvBlock, 2);
    static const uint32_t fill_res = resident_blocks(window_fill_kernel, kWvBlock, 4);
    const uint32_t long_blocks = min((n + kWvWaves - 1) / kWvWaves, long_res);  // up to a wave per unit
    const uint64_t wcap = win_cap(n);
    const uint32_t win_blocks = (uint32_t)std::min<uint64_t>((wcap + kWvWaves - 1) / kWvWaves, spec_res);
    const uint32_t res_blocks = std::min((n + kWvWaves - 1) / kWvWaves, res_res);  // up to a wave per long unit
    const uint32_t wfill_blocks = (uint32_t)std::min<uint64_t>((wcap + kWvWaves - 1) / kWvWaves, fill_res);
    const hipStream_t ss = side.stream();
    long_windows_kernel<<<list_blocks(n), 256, 0, ss>>>(in_len, n, q);
    window_spec_kernel<<<win_blocks, kWvBlock, 0, ss>>>(in, in_off, in_len, n, q);
    window_resolve_kernel<<<res_blocks, kWvBlock, 0, ss>>>(in, in_off, in_len, n, out_cap, out_len, status, q);
    window_fill_kernel<<<wfill_blocks, kWvBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off, status, q);
    decode_wave_kernel<kWvLong><<<long_blocks, kWvBlock, 0, ss>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                   out_len, status, q);
    const uint32_t* const mid = q + kQHead + 2ull * n;
    // the mid units' passes on a second side stream, before the small kernel (mid_side_stream)
    const hipStream_t ms = mid_stream ? side.stream2() : stream;
    if (!mid_stream) {
        if (small_variant() == 0) {
            static const uint32_t sg_res = resident_blocks(decode_small_group_kernel, kSgWaves * kWave, 3);
            decode_small_group_kernel<<<std::min((n + kSgWaves * kWave - 1) / (kSgWaves * kWave), sg_res),
                                        kSgWaves * kWave, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                       out_len, status, q);
        } else {
            decode_small_kernel<<<sm_blocks, kSmBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                     out_len, status, q);
        }
    }
    // mid units: the indexed two-pass decoder (index pass + fill pass), the single-read words
    // decoder, or in a dev build the fused single-pass decoder (capnp_packed_set_decoder)
    if (words) {  // [0, q[20]) two-pass, [q[20], q[4]) words (either may be empty)
        const uint32_t lw_blocks = (n + kLwWaves * kWave - 1) / (kLwWaves * kWave);
        uint8_t* const rec = reinterpret_cast<uint8_t*>(q) + rec_region_off(n);
        decode_index_kernel<false><<<ix_blocks_for(n), kWave * kIxBw, 0, ms>>>(
            in, in_off, in_len, n, out, out_off, out_cap, out_len, status, nullptr, mid, q + 20, rec);
        decode_fill_kernel<<<fill_blocks(n), kFlWaves * kWave, 0, ms>>>(in, in_off, in_len, n, out, out_off,
                                                                           out_len, out_cap, status, mid, q + 20, rec);
        decode_words_kernel<false><<<lw_blocks, kLwWaves * kWave, 0, ms>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                          out_len, status, mid, q + 4, q + 20, q + 21,
                                                                          nullptr);
        // the words decoder's units stopped at their slot's capacity with input left (q[21] of them,
        // usually none: the kernel returns at once)
        decode_wave_kernel<kWvMarked><<<fallback_blocks(n), kWvBlock, 0, ms>>>(in, in_off, in_len, n, out, out_off,
                                                                            out_cap, out_len, status, q + 21);
    } else
    {
        uint8_t* const rec = reinterpret_cast<uint8_t*>(q) + rec_region_off(n);  // piece records, off the output slots
        decode_index_kernel<false><<<ix_blocks_for(n), kWave * kIxBw, 0, ms>>>(
            in, in_off, in_len, n, out, out_off, out_cap, out_len, status, nullptr, mid, q + 4, rec);
        decode_fill_kernel<<<fill_blocks(n), kFlWaves * kWave, 0, ms>>>(in, in_off, in_len, n, out, out_off,
                                                                           out_len, out_cap, status, mid, q + 4, rec);
    }
    if (mid_stream) {
        if (small_variant() == 0) {
            static const uint32_t sg_res = resident_blocks(decode_small_group_kernel, kSgWaves * kWave, 3);
            decode_small_group_kernel<<<std::min((n + kSgWaves * kWave - 1) / (kSgWaves * kWave), sg_res),
                                        kSgWaves * kWave, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                       out_len, status, q);
        } else {
            decode_small_kernel<<<sm_blocks, kSmBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                     out_len, status, q);
        }
    }
    e = hipGetLastError();
    const hipError_t j = side.join();
    return e != hipSuccess ? e : j;
}

hipError_t launch_encode_message(const uint64_t* seg_ptr, const uint64_t* seg_len, const uint32_t* seg_first,
                                 const uint32_t* seg_count, uint32_t n, uint8_t* out, const uint64_t* out_off,
                                 const uint64_t* out_cap, uint64_t* out_len, int32_t* status, bool write,
                                 hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // every message, then the marked multi-tile ones (a grid striding over the statuses)
    const uint32_t tiled_blocks = min(((n + kWave - 1) / kWave + kWavesPerBlock - 1) / kWavesPerBlock, 2048u);
    if (write) {
        encode_message_kernel<true, false><<<blocks_for((n + 1) / 2), kBlock, 0, stream>>>(
                seg_ptr, seg_len, seg_first, seg_count, n, out, out_off, out_cap, out_len, status);
        encode_message_kernel<true, true><<<tiled_blocks, kBlock, 0, stream>>>(
            seg_ptr, seg_len, seg_first, seg_count, n, out, out_off, out_cap, out_len, status);
    } else {
        encode_message_kernel<false, false><<<blocks_for((n + 1) / 2), kBlock, 0, stream>>>(
                seg_ptr, seg_len, seg_first, seg_count, n, out, out_off, out_cap, out_len, status);
        encode_message_kernel<false, true><<<tiled_blocks, kBlock, 0, stream>>>(
            seg_ptr, seg_len, seg_first, seg_count, n, out, out_off, out_cap, out_len, status);
    }
    return hipGetLastError();
}

hipError_t launch_message_init(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                               uint32_t max_segs, uint32_t* seg_count, uint64_t* seg_off, uint64_t* seg_len,
                               int32_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    message_init_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, stream>>>(in, in_off, in_len, n, max_segs,
                                                                          seg_count, seg_off, seg_len, status);
    return hipGetLastError();
}

// Single-buffer calls (one unit, capnp_packed_decode / capnp_packed_encode up to 24 KiB / 4 KiB):
// one kernel instead of the batch sequence (classes, side-stream fork and join, ~12 launches):
// decode by the serial window walk of one wave (decode_wave_kernel<kWvMarked>: all-or-nothing,
// any size, a window of 4.6 KB at a time), encode by the one-tile encoder.
int32_t decode_one_status() { return kStNeedFull; }
hipError_t launch_decode_one(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                             hipStream_t stream) {
    decode_wave_kernel<kWvMarked><<<1, kWvBlock, 0, stream>>>(in, in_off, in_len, 1, out, out_off, out_cap, out_len,
                                                               status, nullptr);
    return hipGetLastError();
}
hipError_t launch_encode_one(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                             bool write, hipStream_t stream) {
    if (write)
        encode_kernel<true><<<1, kBlock, 0, stream>>>(in, in_off, in_len, 1, out, out_off, out_cap, out_len, status,
                                                        nullptr, nullptr);
    else
        encode_kernel<false><<<1, kBlock, 0, stream>>>(in, in_off, in_len, 1, out, out_off, out_cap, out_len, status,
                                                         nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_read_message(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                               uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                               uint64_t* consumed, int32_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    read_header_kernel<true><<<(n + kBlock - 1) / kBlock, kBlock, 0, stream>>>(in, in_off, in_len, n, out_len, consumed,
                                                                        status);
    // messages of more than kRdWordsMax words (kStNeedWalk): the walk to the framed length, then
    // the gated write pass, the fill pass and the fallback (each takes only the statuses it owns)
    decode_index_kernel<true, kRdWalk><<<ix_blocks_for(n), kWave * kIxBw, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                  out_len, status, consumed);
    // the message's own bytes from here on: in_len = consumed
    decode_index_kernel<false, kRdGate><<<ix_blocks_for(n), kWave * kIxBw, 0, stream>>>(in, in_off, consumed, n, out, out_off, out_cap,
                                                                   out_len, status, nullptr);
    decode_fill_kernel<<<fill_blocks(n), kFlWaves * kWave, 0, stream>>>(in, in_off, consumed, n, out, out_off,
                                                                       out_len, out_cap, status);
    decode_wave_kernel<kWvMarked><<<fallback_blocks(n), kWvBlock, 0, stream>>>(in, in_off, consumed, n, out, out_off,
                                                                        out_cap, out_len, status, nullptr);
    // the rest (kStWords): the words decoder, stopped at the framed length; last, so that the fill
    // pass above (it takes OK units) never sees the units it finishes
    decode_words_kernel<true><<<(n + kLwWaves * kWave - 1) / (kLwWaves * kWave), kLwWaves * kWave, 0, stream>>>(
        in, in_off, in_len, n, out, out_off, out_cap, out_len, status, nullptr, nullptr, nullptr, nullptr, consumed);
    return hipGetLastError();
}

hipError_t launch_copy_jobs(const uint64_t* jobs, uint32_t nj, hipStream_t stream) {
    if (nj == 0) return hipSuccess;
    copy_jobs_kernel<<<std::min(nj, 4096u), 256, 0, stream>>>(jobs, nj);
    return hipGetLastError();
}

hipError_t launch_read_header(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                              uint64_t* out_len, uint64_t* consumed, int32_t* status, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    read_header_kernel<false><<<(n + kBlock - 1) / kBlock, kBlock, 0, stream>>>(in, in_off, in_len, n, out_len, consumed,
                                                                         status);
    return hipGetLastError();
}

// The framer's window table: entry g of list connection i's windows names i as its unit and
// its first window (window_spec_kernel's WinEnt.unit / .first).
__global__ __launch_bounds__(256) void framer_windows_kernel(const uint32_t* __restrict__ first,
                                                             const uint32_t* __restrict__ count, uint32_t nl,
                                                             uint32_t* q, uint32_t nq) {
    WinEnt* const tab = win_tab(q, nq);
    for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x)
        for (uint32_t w = threadIdx.x; w < count[i]; w += blockDim.x) {
            tab[first[i] + w].unit = i;
            tab[first[i] + w].first = first[i];
        }
}

size_t framer_spec_bytes(uint32_t nl, uint64_t windows) { return 4 * win_tab_off(nl) + sizeof(WinEnt) * windows; }
uint32_t framer_window_bytes() { return kWvWin; }
uint64_t framer_window_cap(uint32_t nl) { return win_cap(nl); }

hipError_t launch_frame_walk(const uint8_t* arena, const uint32_t* list, uint32_t nl, const uint64_t* base,
                             const uint64_t* avail, uint64_t* need, uint64_t* X, uint64_t* W, int32_t* status,
                             uint32_t M, uint32_t* cnt, uint32_t* tab, uint32_t* spec_q, uint64_t windows,
                             const uint32_t* spec_first, const uint32_t* spec_count, const uint64_t* spec_off,
                             const uint64_t* spec_len, hipStream_t stream) {
    if (nl == 0) return hipSuccess;
    const WinEnt* spec = nullptr;
    if (spec_q && windows) {  // spec tables of every listed connection's windows, in parallel
        framer_windows_kernel<<<std::min(nl, 1024u), 256, 0, stream>>>(spec_first, spec_count, nl, spec_q, nl);
        static const uint32_t spec_res = resident_blocks(window_spec_kernel, kWvBlock, 4);
        const uint32_t sb = (uint32_t)std::min<uint64_t>((windows + kWvWaves - 1) / kWvWaves, spec_res);
        window_spec_kernel<<<sb, kWvBlock, 0, stream>>>(arena, spec_off, spec_len, nl, spec_q);
        spec = reinterpret_cast<const WinEnt*>(spec_q + win_tab_off(nl));
    }
    static const uint32_t res = resident_blocks(frame_walk_kernel, kWvBlock, 2);
    const uint32_t blocks = std::min((nl + kWvWaves - 1) / kWvWaves, res);
    frame_walk_kernel<<<blocks, kWvBlock, 0, stream>>>(arena, list, nl, base, avail, need, X, W, status, spec,
                                                        spec ? spec_first : nullptr, M, cnt, tab);
    return hipGetLastError();
}

hipError_t launch_validate(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                           uint64_t seg_limit, uint64_t trav_limit, uint32_t nest_limit, int32_t* status,
                           uint64_t* words, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // persistent grid: the resident waves, each owning a contiguous range of messages
    static const uint32_t resident = [] {  // thread-safe one-time init (C++11 static)
        int dev = 0, cus = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, validate_kernel<false>, kWave, 0) != hipSuccess || per <= 0)
            per = 8;
        return (uint32_t)(cus * per);
    }();
    const uint32_t full = (n + kWave - 1) / kWave;
    const uint32_t blocks = full < resident ? full : resident;
    const uint32_t per_wave = (uint32_t)(((uint64_t)n + blocks - 1) / blocks);
    if (nest_limit > kVdMaxNest) nest_limit = kVdMaxNest;
    VdDeep dp;
    const bool deep = nest_limit > kVdDepth;
    void* lst = nullptr;
    if (deep) {  // messages needing more than 64 frames go to a list for the DEEP kernel
        hipError_t e = hipMallocAsync(&lst, 4ull * n + 16, stream);
        if (e == hipSuccess) e = hipMemsetAsync(lst, 0, 16, stream);
        if (e != hipSuccess) return e;
        dp.count = static_cast<uint32_t*>(lst);
        dp.list = dp.count + 4;
    }
    validate_kernel<false><<<blocks, kWave, 0, stream>>>(in, in_off, in_len, n, per_wave, seg_limit, trav_limit,
                                                         nest_limit, status, words, dp);
    if (!deep) return hipGetLastError();
    // Frames of the DEEP kernel: a message holds at most min(nesting_limit, traversal limit)
    // of them (each spends a nesting level and at least one traversal word); lanes sized so
    // the stacks take at most kVdDeepBytes (at least one lane), at most 64 waves.
    constexpr uint64_t kVdDeepBytes = 256ull << 20;
    const uint64_t cap = trav_limit < nest_limit ? (trav_limit ? trav_limit : 1) : nest_limit;
    const uint64_t per_lane = cap * (sizeof(uint4) + sizeof(uint32_t));
    uint64_t lanes = kVdDeepBytes / per_lane;
    lanes = lanes < 1 ? 1 : lanes > 64ull * kWave ? 64ull * kWave : lanes;
    void* stk = nullptr;
    hipError_t e = hipMallocAsync(&stk, lanes * per_lane, stream);
    if (e != hipSuccess) {
        (void)hipFreeAsync(lst, stream);
        return e;
    }
    dp.stk = static_cast<uint4*>(stk);
    dp.nest = reinterpret_cast<uint32_t*>(dp.stk + lanes * cap);
    dp.depth_cap = (uint32_t)cap;
    dp.lanes = (uint32_t)lanes;
    validate_kernel<true><<<(uint32_t)((lanes + kWave - 1) / kWave), kWave, 0, stream>>>(
        in, in_off, in_len, n, 0, seg_limit, trav_limit, nest_limit, status, words, dp);
    e = hipGetLastError();
    (void)hipFreeAsync(stk, stream);
    (void)hipFreeAsync(lst, stream);
    return e;
}

hipError_t launch_generate(uint8_t* out, uint64_t n_units, uint64_t unit_bytes, uint64_t unit_base,
                           uint64_t seed, uint32_t thr, hipStream_t stream) {
    const uint64_t total = n_units * (unit_bytes / 8);
    if (total == 0) return hipSuccess;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    generate_kernel<<<(uint32_t)blocks, 256, 0, stream>>>(out, n_units, unit_bytes / 8, unit_base, seed, thr);
    return hipGetLastError();
}

size_t scan_scratch_bytes(uint32_t n) {
    return ((size_t)(n + kScanTile - 1) / kScanTile + 1) * sizeof(uint64_t);
}

hipError_t launch_scan(const uint64_t* len, uint32_t n, uint64_t base, uint64_t* off, uint64_t* scratch,
                       hipStream_t stream) {
    const uint32_t nb = (n + kScanTile - 1) / kScanTile;
    if (n == 0) {
        scan_partials_kernel<<<1, 1024, 0, stream>>>(scratch, 0, base, off, 0);
        return hipGetLastError();
    }
    scan_local_kernel<<<nb, 256, 0, stream>>>(len, n, off, scratch);
    scan_partials_kernel<<<1, 1024, 0, stream>>>(scratch, nb, base, off, n);
    scan_apply_kernel<<<nb, 256, 0, stream>>>(off, n, scratch);
    return hipGetLastError();
}

}  // namespace cpk

// Diagnostic builds only: read and clear the phase cycle sums.

