// packed_kernels.hip — CDNA4 (gfx950) kernels for the Cap'n Proto packed codec.
//
// Reference semantics (Zig rules, NOT canonical C++ capnp):
//   encode  nullstyle/capnp-zig src/serialization/message.zig:200-271 (packPacked)
//   decode  message.zig:88-145 (unpackPacked) with the size pass of :152-191
//
// Execution model: one 64-lane wave owns one unit (one packPacked
// / unpackPacked call). A unit is staged in the wave's private LDS slice with
// coalesced 16-B global loads, processed with wave-wide scans, assembled in LDS
// and written back with coalesced 16-B stores. No MFMA: this is byte compaction.
//
//   encode: lane j owns words [8j, 8j+8). Each word's zero-byte tag is formed
//           with SWAR + a multiply gather; zero/literal runs (greedy, 256-capped)
//           are resolved with wave max/min scans of break positions; a wave sum
//           scan gives every lane its output byte offset; each lane appends its
//           records to a byte stream in LDS (u64 ds_or at 8-B granularity).
//   decode: the record chain (tag -> record length) is serial. Lanes walk
//           64-byte chunks of the staged packed bytes speculatively from the
//           chunk start; a fix-up loop re-walks lanes whose true entry point is
//           not on their speculative chain (walks couple after a few records,
//           so 1-2 rounds are typical, 64 worst case). Record starts become one
//           u64 bitmask per lane; a wave sum scan of words-per-record gives
//           output word offsets; mixed words are expanded with v_perm_b32 and a
//           selector LUT; zero runs cost nothing (the LDS window is pre-zeroed).
//
// Units larger than the fast-path limits run a serial per-wave path (lane 0)
// that reads and writes global memory directly (correct for any size; slow).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

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

// ---- decode fast path ------------------------------------------------------
constexpr uint32_t kDecIn = 4864;                      // staged packed bytes
constexpr uint32_t kDecPMax = kDecIn - 16 - 32;        // 4816 B of packed input per unit
constexpr uint32_t kDecWinWords = 512;                 // output window (words)
constexpr uint32_t kDecOut = kDecWinWords * 8 + 16;    // 4112 B

enum : int32_t {
    ST_OK = CAPNP_PACKED_OK,
    ST_SIZE = CAPNP_PACKED_INVALID_MESSAGE_SIZE,
    ST_EOF = CAPNP_PACKED_UNEXPECTED_EOF,
    ST_SPACE = CAPNP_PACKED_OUT_OF_SPACE,
    ST_ARG = CAPNP_PACKED_INVALID_ARGUMENT,
};

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------

// Order LDS traffic between lanes of ONE wave (the wave owns its LDS slice).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t t = __shfl_up(v, d, kWave);
        if (lane >= (uint32_t)d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t t = __shfl_up(v, d, kWave);
        if (lane >= (uint32_t)d) v = max(v, t);
    }
    return v;
}

// inclusive min over lanes >= this lane
__device__ __forceinline__ uint32_t wave_incl_suffix_min(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t t = __shfl_down(v, d, kWave);
        if (lane + d < (uint32_t)kWave) v = min(v, t);
    }
    return v;
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
    return nonzero_tag32((uint32_t)w) | (nonzero_tag32((uint32_t)(w >> 32)) << 4);
}

// v_perm_b32 over the 8 bytes of d: selector byte r in 0..7 picks byte r, 0x0C gives 0.
__device__ __forceinline__ uint64_t perm64(uint64_t d, uint64_t sel) {
    uint32_t lo = (uint32_t)d, hi = (uint32_t)(d >> 32);
    uint32_t a = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
    uint32_t b = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
    return (uint64_t)a | ((uint64_t)b << 32);
}

// Selector that gathers the nonzero bytes of a word with tag t into bytes 0..popc-1.
__device__ inline uint64_t compact_selector(uint32_t t) {
    uint64_t sel = 0x0C0C0C0C0C0C0C0CULL;
    int r = 0;
    for (int k = 0; k < 8; ++k) {
        if ((t >> k) & 1u) {
            sel = (sel & ~(0xFFULL << (8 * r))) | ((uint64_t)k << (8 * r));
            ++r;
        }
    }
    return sel;
}

// Selector that scatters popc(t) packed bytes back to the set-bit positions of t.
__device__ inline uint64_t expand_selector(uint32_t t) {
    uint64_t sel = 0;
    int r = 0;
    for (int k = 0; k < 8; ++k) {
        uint64_t s = 0x0C;
        if ((t >> k) & 1u) s = (uint64_t)(r++);
        sel |= s << (8 * k);
    }
    return sel;
}

// Unaligned 8-byte read from an LDS byte array (two aligned ds_read_b64 + funnel).
__device__ __forceinline__ uint64_t lds_read_u64_unaligned(const uint8_t* base, uint32_t p) {
    uint32_t a = p & ~7u;
    uint64_t lo = *reinterpret_cast<const uint64_t*>(base + a);
    uint64_t hi = *reinterpret_cast<const uint64_t*>(base + a + 8);
    uint32_t sh = (p & 7u) * 8u;
    return sh ? ((lo >> sh) | (hi << (64u - sh))) : lo;
}

// Stage nch 16-B chunks from global g[0 .. 16*nch) into lds[0 .. 16*nch):
// lane l moves chunks l, l+64, ... All K loads are issued before the first LDS
// store (addresses clamped to the last chunk, guards wave-uniform) so they stay
// in VGPRs and overlap in flight.
template <int K>
__device__ __forceinline__ void stage_linear(uint8_t* lds, const uint8_t* g, uint32_t nch, uint32_t lane) {
    if (nch == 0) return;
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {  // unconditional: clamped lanes re-read the last chunk (same line)
        uint32_t c = min(lane + 64u * k, nch - 1);
        v[k] = *reinterpret_cast<const uint4*>(g + 16 * (uint64_t)c);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t c = lane + 64u * k;
        if ((uint32_t)(64 * k) < nch && c < nch) *reinterpret_cast<uint4*>(lds + 16 * c) = v[k];
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

// Per-lane byte stream into a zero-initialised LDS buffer. Every flushed u64 is
// OR-ed (ds_or_b64) so the partial words a lane shares with its neighbours merge.
struct LdsByteStream {
    uint8_t* lds;
    uint32_t addr;  // 8-aligned byte address of acc
    uint32_t fill;  // bytes already in acc (0..7)
    uint64_t acc;

    __device__ __forceinline__ void init(uint8_t* base, uint32_t start) {
        lds = base;
        addr = start & ~7u;
        fill = start & 7u;
        acc = 0;
    }
    __device__ __forceinline__ void flush(uint64_t v) {
        atomicOr(reinterpret_cast<unsigned long long*>(lds + addr), (unsigned long long)v);
    }
    // append k (<= 8) bytes held in the low bytes of v (bytes >= k must be zero)
    __device__ __forceinline__ void put(uint64_t v, uint32_t k) {
        if (k == 0) return;
        uint32_t sh = fill * 8u;
        uint64_t a = fill ? (acc | (v << sh)) : v;
        uint32_t nf = fill + k;
        if (nf >= 8) {
            flush(a);
            addr += 8;
            acc = fill ? (v >> (64u - sh)) : 0;
            fill = nf - 8;
        } else {
            acc = a;
            fill = nf;
        }
    }
    __device__ __forceinline__ void finish() {
        if (fill) flush(acc);
    }
};

// ---------------------------------------------------------------------------
// Serial per-wave fallback (lane 0), any unit size. Restates message.zig
// directly over global memory. Used for units beyond the fast-path limits.
// ---------------------------------------------------------------------------

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
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void encode_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint64_t* __restrict__ in_len,
                                                        uint32_t n, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint64_t* __restrict__ out_cap,
                                                        uint64_t* __restrict__ out_len,
                                                        int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * (WRITE ? kEncLds : kEncLds)];
    __shared__ uint64_t lut[256];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (WRITE) {
        lut[threadIdx.x] = compact_selector(threadIdx.x);
        __syncthreads();
    }
    const uint32_t unit = blockIdx.x * kWavesPerBlock + wave;
    if (unit >= n) return;
    uint8_t* lds = smem + wave * kEncLds;

    const uint64_t b0 = in_off[unit];
    const uint64_t nbytes = in_len[unit];
    uint64_t ob = 0, cap = 0;
    int32_t st = ST_OK;
    if (WRITE) {
        ob = out_off[unit];
        cap = out_cap[unit];
    }
    if (reinterpret_cast<uintptr_t>(in + b0) & 7) st = ST_ARG;
    if (st == ST_OK && (nbytes & 7)) st = ST_SIZE;  // message.zig:201
    if (st != ST_OK) {
        if (lane == 0) { out_len[unit] = 0; status[unit] = st; }
        return;
    }
    if (nbytes / 8 > kEncMaxWords) {
        // serial fallback
        if (lane == 0) {
            uint64_t P = serial_pack(in + b0, nbytes / 8, nullptr);
            int32_t s2 = ST_OK;
            if (WRITE) {
                if (P > cap) s2 = ST_SPACE;
                else serial_pack(in + b0, nbytes / 8, out + ob);
            }
            out_len[unit] = P;
            status[unit] = s2;
        }
        return;
    }
    const uint32_t words = (uint32_t)(nbytes >> 3);

    // ---- stage the unit into LDS, word w at row (w>>3)*80 + (w&7)*8 ------------
    {
        const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(in + b0) & 15);  // 0 or 8
        const uint8_t* g = in + b0 - s;
        const uint32_t nch = (s + (uint32_t)nbytes + 15) >> 4;
        uint4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if ((uint32_t)(64 * k) < nch) {
                uint32_t c = min(lane + 64u * k, nch - 1);
                v[k] = *reinterpret_cast<const uint4*>(g + 16 * (uint64_t)c);
            }
        }
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
    wave_lds_sync();

    // ---- lane j owns words [8j, 8j+8) ------------------------------------------
    const uint32_t base = lane * 8;
    const uint32_t nw = base < words ? min(8u, words - base) : 0u;
    uint64_t w[8];
    if (nw) {
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
        if ((uint32_t)t < nw) {
            if (tag[t] == 0) zmask |= 1u << t;
            if (tag[t] == 0xFF) fmask |= 1u << t;
        }
    }
    // break positions for the zero-run (Z) and literal-run (F) classes
    uint32_t lbz = 0, lbf = 0, fbz = words, fbf = words;
#pragma unroll
    for (int t = 7; t >= 0; --t) {
        uint32_t i = base + t;
        if (!((zmask >> t) & 1u)) { lbz = max(lbz, i + 1); fbz = i; }
        if (!((fmask >> t) & 1u)) { lbf = max(lbf, i + 1); fbf = i; }
    }
    fbz = min(fbz, words);
    fbf = min(fbf, words);
    // run start carried into this lane = last break before it (+1); run end = first break after it
    uint32_t cz = __shfl_up(wave_incl_max(lbz, lane), 1, kWave);
    uint32_t cf = __shfl_up(wave_incl_max(lbf, lane), 1, kWave);
    uint32_t ez = __shfl_down(wave_incl_suffix_min(fbz, lane), 1, kWave);
    uint32_t ef = __shfl_down(wave_incl_suffix_min(fbf, lane), 1, kWave);
    if (lane == 0) { cz = 0; cf = 0; }
    if (lane == 63) { ez = words; ef = words; }
    ez = min(ez, words);
    ef = min(ef, words);

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
        if (!((zmask >> t) & 1u)) ez = i;
        if (!((fmask >> t) & 1u)) ef = i;
    }
    uint32_t sz[8], cnt[8];
    uint32_t total = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        uint32_t i = base + t;
        uint32_t head = ((i - rs[t]) & 255u) == 0;
        cnt[t] = min(256u, re[t] - i) - 1;  // message.zig:214-223 / 236-245
        uint32_t s;
        if ((uint32_t)t >= nw) s = 0;
        else if ((zmask >> t) & 1u) s = head ? 2 : 0;
        else if ((fmask >> t) & 1u) s = head ? 10 : 8;
        else s = 1 + __popc(tag[t]);
        sz[t] = s;
        total += s;
    }
    const uint32_t incl = wave_incl_sum(total, lane);
    const uint32_t P = readlane(incl, 63);
    const uint32_t o = incl - total;

    if (!WRITE) {
        if (lane == 0) { out_len[unit] = P; status[unit] = ST_OK; }
        return;
    }
    if ((uint64_t)P > cap) {
        if (lane == 0) { out_len[unit] = P; status[unit] = ST_SPACE; }
        return;
    }

    // ---- assemble the packed bytes in LDS (reusing the staging slice) -------------
    const uint32_t so = (uint32_t)(reinterpret_cast<uintptr_t>(out + ob) & 15);
    const uint32_t nch_out = (so + P + 15) >> 4;
    wave_lds_sync();  // every lane has its words in registers
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        uint32_t c = lane + 64 * k;
        if (c < nch_out) *reinterpret_cast<uint4*>(lds + 16 * c) = make_uint4(0, 0, 0, 0);
    }
    wave_lds_sync();
    {
        LdsByteStream bs;
        bs.init(lds, so + o);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (sz[t] == 0) continue;
            if ((zmask >> t) & 1u) {
                bs.put((uint64_t)cnt[t] << 8, 2);                       // 00 <count>
            } else if ((fmask >> t) & 1u) {
                if (sz[t] == 10) {                                       // FF w0..w7 <count>
                    bs.put(0xFFULL | (w[t] << 8), 8);
                    bs.put((w[t] >> 56) | ((uint64_t)cnt[t] << 8), 2);
                } else {
                    bs.put(w[t], 8);                                     // literal run body
                }
            } else {                                                     // tag + nonzero bytes
                uint64_t comp = perm64(w[t], lut[tag[t]]);
                bs.put((uint64_t)tag[t] | (comp << 8), sz[t]);
            }
        }
        bs.finish();
    }
    wave_lds_sync();

    // ---- coalesced write-back ------------------------------------------------------
    {
        uint8_t* gdst = out + ob - so;  // 16-B aligned
        const uint32_t lo = so, hi = so + P;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint32_t c = lane + 64 * k;
            if (c < nch_out) {
                uint32_t cb = 16 * c, ce = cb + 16;
                if (cb >= lo && ce <= hi) {
                    *reinterpret_cast<uint4*>(gdst + cb) = *reinterpret_cast<const uint4*>(lds + cb);
                } else {
                    uint32_t a = max(cb, lo), e = min(ce, hi);
                    for (uint32_t b = a; b < e; ++b) gdst[b] = lds[b];
                }
            }
        }
    }
    if (lane == 0) { out_len[unit] = P; status[unit] = ST_OK; }
}

// ---------------------------------------------------------------------------
// DECODE
// ---------------------------------------------------------------------------

// Walk record starts of one 64-byte chunk [cs, ce) from entry e.
// Record length: 00 -> 2, FF -> 10 + 8*count, other -> 1 + popc(tag)  (message.zig:152-191)
__device__ __forceinline__ void walk_chunk(const uint8_t* lds, uint32_t e, uint32_t cs, uint32_t ce,
                                           uint64_t& mask, uint32_t& exit_pos) {
    uint32_t pos = e;
    uint64_t m = 0;
    while (pos < ce) {
        m |= 1ULL << (pos - cs);
        uint32_t t = lds[pos];
        uint32_t len = (t == 0) ? 2u : (t == 0xFF ? 10u + 8u * (uint32_t)lds[pos + 9] : 1u + __popc(t));
        pos += len;
    }
    mask = m;
    exit_pos = pos;
}

template <bool WRITE>
__global__ __launch_bounds__(kBlock) void decode_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint64_t* __restrict__ in_len,
                                                        uint32_t n, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint64_t* __restrict__ out_cap,
                                                        uint64_t* __restrict__ out_len,
                                                        int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kWavesPerBlock * kDecIn];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[kWavesPerBlock * (WRITE ? kDecOut : 16)];
    __shared__ uint64_t lut[256];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (WRITE) {
        lut[threadIdx.x] = expand_selector(threadIdx.x);
        __syncthreads();
    }
    const uint32_t unit = blockIdx.x * kWavesPerBlock + wave;
    if (unit >= n) return;
    uint8_t* lin = s_in + wave * kDecIn;
    uint8_t* lout = s_out + wave * (WRITE ? kDecOut : 16);

    const uint64_t b0 = in_off[unit];
    uint64_t ob = 0, cap = 0;
    int32_t st = ST_OK;
    if (WRITE) {
        ob = out_off[unit];
        cap = out_cap[unit];
        if (reinterpret_cast<uintptr_t>(out + ob) & 7) st = ST_ARG;
    }
    if (st != ST_OK) {
        if (lane == 0) { out_len[unit] = 0; status[unit] = st; }
        return;
    }
    const uint64_t P64 = in_len[unit];
    if (P64 > kDecPMax) {
        if (lane == 0) {
            uint64_t U = 0;
            int32_t s2 = serial_decoded_size(in + b0, P64, &U);
            if (s2 != ST_OK) U = 0;
            else if (WRITE) {
                if (U > cap) s2 = ST_SPACE;
                else serial_unpack(in + b0, P64, out + ob);
            }
            out_len[unit] = U;
            status[unit] = s2;
        }
        return;
    }
    const uint32_t P = (uint32_t)P64;
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(in + b0) & 15);
    const uint32_t end = s + P;

    // ---- stage packed bytes (16-B aligned chunks; bytes outside [s, end) are ignored)
    stage_linear<5>(lin, in + b0 - s, (end + 15) >> 4, lane);
    wave_lds_sync();

    // ---- record discovery: speculative chunk walks + fix-up ---------------------------
    const uint32_t nc = (P + 63) >> 6;  // 64-byte chunks (<= 76)
    uint64_t m[2] = {0, 0};
    uint32_t carry = s;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        if ((uint32_t)(64 * r) >= nc) break;
        const uint32_t c = 64 * r + lane;
        const bool active = c < nc;
        const uint32_t cs = s + 64 * c;
        const uint32_t ce = min(cs + 64, end);
        uint64_t mask = 0;
        uint32_t ex = cs;
        if (active) walk_chunk(lin, lane == 0 ? carry : cs, cs, ce, mask, ex);
        uint32_t entry = carry;
        for (int it = 0; it < 66; ++it) {
            uint32_t prev = __shfl_up(ex, 1, kWave);
            entry = (lane == 0) ? carry : prev;
            bool ok = true;
            if (active) {
                if (entry >= ce) ok = (mask == 0 && ex == entry);
                else ok = (entry >= cs) && ((mask >> (entry - cs)) & 1ULL);
            }
            if (__all(ok)) break;
            if (!ok) walk_chunk(lin, entry, cs, ce, mask, ex);
        }
        if (active && entry < ce && entry > cs) mask &= ~0ULL << (entry - cs);
        m[r] = mask;
        const uint32_t last = min(nc - 64 * r, 64u) - 1;
        carry = readlane(ex, last);
    }
    const bool eof = (carry != end);  // the record chain must end exactly at the last byte

    // ---- words per lane, output word offsets ----------------------------------------
    uint32_t wc[2] = {0, 0};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        uint64_t bits = m[r];
        const uint32_t cs = s + 64 * (64 * r + lane);
        while (bits) {
            uint32_t b = __builtin_ctzll(bits);
            bits &= bits - 1;
            uint32_t pos = cs + b;
            uint32_t t = lin[pos];
            wc[r] += (t == 0) ? 1u + lin[pos + 1] : (t == 0xFF ? 1u + lin[pos + 9] : 1u);
        }
    }
    const uint32_t inc0 = wave_incl_sum(wc[0], lane);
    const uint32_t tot0 = readlane(inc0, 63);
    const uint32_t inc1 = wave_incl_sum(wc[1], lane);
    const uint32_t W = tot0 + readlane(inc1, 63);
    const uint32_t wbase[2] = {inc0 - wc[0], tot0 + inc1 - wc[1]};

    if (eof) {
        if (lane == 0) { out_len[unit] = 0; status[unit] = ST_EOF; }
        return;
    }
    const uint64_t U = 8ULL * W;
    if (!WRITE) {
        if (lane == 0) { out_len[unit] = U; status[unit] = ST_OK; }
        return;
    }
    if (U > cap) {
        if (lane == 0) { out_len[unit] = U; status[unit] = ST_SPACE; }
        return;
    }

    // ---- expansion, one 512-word output window at a time -------------------------------
    const uint32_t so = (uint32_t)(reinterpret_cast<uintptr_t>(out + ob) & 15);  // 0 or 8
    for (uint32_t win = 0; win < W; win += kDecWinWords) {
        const uint32_t nwin = min(kDecWinWords, W - win);
        const uint32_t nbytes = so + 8 * nwin;
        const uint32_t nch = (nbytes + 15) >> 4;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint32_t c = lane + 64 * k;
            if (c < nch) *reinterpret_cast<uint4*>(lout + 16 * c) = make_uint4(0, 0, 0, 0);
        }
        wave_lds_sync();
        const uint32_t wend = win + nwin;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            uint64_t bits = m[r];
            const uint32_t cs = s + 64 * (64 * r + lane);
            uint32_t wo = wbase[r];
            while (bits && wo < wend) {
                uint32_t b = __builtin_ctzll(bits);
                bits &= bits - 1;
                uint32_t pos = cs + b;
                uint32_t t = lin[pos];
                if (t == 0) {
                    wo += 1u + lin[pos + 1];                         // zero run: window is pre-zeroed
                } else if (t == 0xFF) {
                    uint32_t c = lin[pos + 9];
                    uint32_t k0 = wo < win ? win - wo : 0u;
                    uint32_t k1 = min(c + 1, wend - wo);
                    for (uint32_t k = k0; k < k1; ++k) {
                        uint32_t src = k == 0 ? pos + 1 : pos + 10 + 8 * (k - 1);
                        *reinterpret_cast<uint64_t*>(lout + so + 8 * (wo + k - win)) =
                            lds_read_u64_unaligned(lin, src);
                    }
                    wo += 1 + c;
                } else {
                    if (wo >= win) {
                        uint64_t d = lds_read_u64_unaligned(lin, pos + 1);
                        *reinterpret_cast<uint64_t*>(lout + so + 8 * (wo - win)) = perm64(d, lut[t]);
                    }
                    wo += 1;
                }
            }
        }
        wave_lds_sync();
        uint8_t* gdst = out + ob + 8ULL * win - so;  // 16-B aligned
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint32_t c = lane + 64 * k;
            if (c < nch) {
                uint32_t cb = 16 * c;
                if (cb >= so && cb + 16 <= nbytes) {
                    *reinterpret_cast<uint4*>(gdst + cb) = *reinterpret_cast<const uint4*>(lout + cb);
                } else {  // one valid 8-byte half
                    uint32_t h = cb < so ? cb + 8 : cb;
                    *reinterpret_cast<uint64_t*>(gdst + h) = *reinterpret_cast<const uint64_t*>(lout + h);
                }
            }
        }
        wave_lds_sync();
    }
    if (lane == 0) { out_len[unit] = U; status[unit] = ST_OK; }
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

template <bool WRITE>
__global__ __launch_bounds__(kBlock) void decode_lane_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ in_off,
                                                             const uint64_t* __restrict__ in_len,
                                                             uint32_t n, uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off,
                                                             const uint64_t* __restrict__ out_cap,
                                                             uint64_t* __restrict__ out_len,
                                                             int32_t* __restrict__ status) {
    __shared__ uint64_t lut[256];
    if (WRITE) {
        lut[threadIdx.x] = expand_selector(threadIdx.x);
        __syncthreads();
    }
    const uint32_t unit = blockIdx.x * kBlock + threadIdx.x;
    if (unit >= n) return;
    const uint8_t* src = in + in_off[unit];
    const uint64_t P = in_len[unit];
    uint64_t* dst = nullptr;
    uint64_t capw = 0;
    if (WRITE) {
        uint8_t* o = out + out_off[unit];
        if (reinterpret_cast<uintptr_t>(o) & 7) {
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
// DECODE, lane per unit, lockstep output rounds (the production decoder)
// ---------------------------------------------------------------------------
// Lane l of a wave owns unit wave_base + l and walks its record chain exactly
// once (input side: per-lane register window, as in decode_lane_kernel). The
// OUTPUT side is made regular: in every round each live lane emits exactly
// kRoundWords words (one 128-B line) into its row of an LDS ring; zero runs and
// literal runs that cross a round boundary carry over as pending counts. After
// each round the wave stores the ring cooperatively: 8 lanes per 128-B line,
// 8 lines per store instruction (fully coalesced), instead of 64 scattered
// 8-byte stores per instruction.
constexpr int kRoundWords = 16;                 // 128 B of output per lane per round
constexpr int kRingRow = kRoundWords * 8 + 16;  // 144 B: 16-B aligned, staggers LDS banks
constexpr int kStreamWaves = 2;                 // waves per block
constexpr int kStreamBlock = kStreamWaves * kWave;

template <uint32_t PF>
__global__ __launch_bounds__(kStreamBlock) void decode_stream_kernel(const uint8_t* __restrict__ in,
                                                                     const uint64_t* __restrict__ in_off,
                                                                     const uint64_t* __restrict__ in_len,
                                                                     uint32_t n, uint8_t* __restrict__ out,
                                                                     const uint64_t* __restrict__ out_off,
                                                                     const uint64_t* __restrict__ out_cap,
                                                                     uint64_t* __restrict__ out_len,
                                                                     int32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[kStreamWaves * kWave * kRingRow];
    __shared__ uint32_t pf_sink[kStreamWaves * kWave];  // LDS-DMA prefetch target, never read
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* ring = ring_all + wave * (kWave * kRingRow);
    const uint32_t unit = (blockIdx.x * kStreamWaves + wave) * kWave + lane;
    const bool valid = unit < n;

    // ---- per-lane unit state -------------------------------------------------------
    const uint8_t* src = in;
    uint64_t P = 0, capw = 0;
    uint8_t* dstb = out;
    int32_t st = ST_OK;
    if (valid) {
        src = in + in_off[unit];
        P = in_len[unit];
        dstb = out + out_off[unit];
        capw = out_cap[unit] >> 3;
        if (reinterpret_cast<uintptr_t>(dstb) & 7) st = ST_ARG;
    }
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    const uint64_t end64 = valid ? s + P : 0;
    const uint8_t* base = src - s;
    const uint32_t npieces = (uint32_t)((end64 + 15) >> 4);
    uint64_t q0, q1, q2, q3, n0, n1;
    uint32_t wb = 0;
    load_piece(base, npieces, 0, q0, q1);
    load_piece(base, npieces, 1, q2, q3);
    load_piece(base, npieces, 2, n0, n1);
    uint32_t* sink = pf_sink + wave * kWave;
    auto ensure = [&](uint32_t p) {
        while (p - wb >= 16) {
            q0 = q2; q1 = q3; q2 = n0; q3 = n1;
            wb += 16;
            load_piece(base, npieces, (wb >> 4) + 2, n0, n1);
            if (PF) {  // pull the line PF bytes ahead into L2 (LDS-DMA into a sink: no VGPR, no wait)
                const uint32_t pa = wb + PF;
                if ((pa & 127) == 0 && pa < npieces * 16) {
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + pa),
                                                     (__attribute__((address_space(3))) void*)sink, 4, 0, 0);
                }
            }
        }
    };
    if (PF) {  // warm the first PF bytes
        for (uint32_t pa = 128; pa < PF && pa < npieces * 16; pa += 128)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + pa),
                                             (__attribute__((address_space(3))) void*)sink, 4, 0, 0);
    }
    uint64_t pos = s;          // next tag
    uint64_t lit = 0;          // next literal word (valid while pend_lit)
    uint32_t pend_zero = 0, pend_lit = 0;
    uint64_t wo = 0;           // words emitted so far
    bool live = valid && st == ST_OK;

    uint64_t* myrow = reinterpret_cast<uint64_t*>(ring + lane * kRingRow);
    while (__any(live)) {
        // ---- one round: each live lane emits up to kRoundWords words -----------------
        uint32_t nw = 0;
#pragma unroll 2
        for (int k = 0; k < kRoundWords; ++k) {
            if (!live) break;
            uint64_t word = 0;
            bool have = true;
            if (pend_zero) {
                --pend_zero;
            } else if (pend_lit) {
                ensure((uint32_t)lit);
                word = view_word8(q0, q1, q2, q3, (uint32_t)lit - wb);
                lit += 8;
                --pend_lit;
            } else if (pos < end64) {
                ensure((uint32_t)pos);
                const uint32_t o = (uint32_t)pos - wb;
                const uint32_t t = view_byte(q0, q1, q2, q3, o);
                if (t == 0x00) {  // message.zig:101-110
                    if (pos + 2 > end64) { st = ST_EOF; have = false; }
                    else { pend_zero = view_byte(q0, q1, q2, q3, o + 1); pos += 2; }
                } else if (t == 0xFF) {  // message.zig:112-128
                    if (pos + 10 > end64) { st = ST_EOF; have = false; }
                    else {
                        const uint32_t c = view_byte(q0, q1, q2, q3, o + 9);
                        if (pos + 10 + 8ULL * c > end64) { st = ST_EOF; have = false; }
                        else {
                            word = view_word8(q0, q1, q2, q3, o + 1);
                            pend_lit = c;
                            lit = pos + 10;
                            pos += 10 + 8ULL * c;
                        }
                    }
                } else {  // message.zig:131-141
                    const uint32_t kk = __popc(t);
                    if (pos + 1 + kk > end64) { st = ST_EOF; have = false; }
                    else {
                        word = expand_word(view_word8(q0, q1, q2, q3, o + 1), t);
                        pos += 1 + kk;
                    }
                }
            } else {
                have = false;  // unit finished
            }
            if (!have) { live = false; break; }
            myrow[nw++] = word;
        }
        wave_lds_sync();
        // ---- cooperative store: lane L moves 16 B of unit row (L>>3)+8j ---------------
        const uint64_t wo_round = wo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t r = (lane >> 3) + 8 * j;  // ring row (= lane of the owning unit)
            const uint32_t i = lane & 7;             // 16-B piece within the row
            const uint32_t rnw = __shfl(nw, r, kWave);
            const uint64_t rwo = __shfl(wo_round, r, kWave);
            const uint64_t rcap = __shfl(capw, r, kWave);
            uint8_t* rdst = reinterpret_cast<uint8_t*>(__shfl(reinterpret_cast<uint64_t>(dstb), r, kWave));
            const uint32_t w0 = 2 * i;  // first word of this piece
            if (w0 < rnw) {
                const uint8_t* rp = ring + r * kRingRow + 16 * i;
                const uint64_t g = rwo + w0;  // unit word index
                uint8_t* gp = rdst + 8 * g;
                const bool both = (w0 + 1 < rnw) && (g + 1 < rcap);
                if (g < rcap) {
                    if (both && !(reinterpret_cast<uintptr_t>(gp) & 15)) {
                        *reinterpret_cast<uint4*>(gp) = *reinterpret_cast<const uint4*>(rp);
                    } else {
                        *reinterpret_cast<uint64_t*>(gp) = *reinterpret_cast<const uint64_t*>(rp);
                        if (both) *reinterpret_cast<uint64_t*>(gp + 8) = *reinterpret_cast<const uint64_t*>(rp + 8);
                    }
                }
            }
        }
        wo += nw;
        wave_lds_sync();
    }
    if (PF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no prefetch may land after the wave exits
    if (!valid) return;
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    out_len[unit] = 8 * wo;
    status[unit] = (wo > capw) ? ST_SPACE : ST_OK;
}

// ---------------------------------------------------------------------------
// DECODE, lane per unit, LDS-DMA input ring + lockstep output rounds
// ---------------------------------------------------------------------------
// Input side: each lane's packed bytes stream through a per-lane ring of
// kSlots 64-byte chunks in LDS, filled by LDS-DMA (global_load_lds_dwordx4: no
// VGPR destination, so nothing forces a wait at issue). Chunks are issued at
// round ends as soon as the slot they reuse is consumed, so every lane keeps
// ~3 chunks (~192 B) in flight; one s_waitcnt per round end lands them. Within
// a DMA instruction, 4 lanes move the 4 x 16 B of one lane's chunk; the 16-B
// pieces are XOR-swizzled by lane so lanes reading the same logical offset hit
// different LDS banks (swizzle applied to the DMA source, read with the same
// swizzle: linear destination).
// Output side: as decode_stream_kernel (lockstep 16-word rounds, cooperative
// 128-B line stores).
template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
struct DmaCfg {
    static constexpr uint32_t kPieces = CHUNK / 16;                // 16-B pieces per lane chunk
    static constexpr uint32_t kTasks = kWave / kPieces;            // lanes whose chunk one DMA moves
    static constexpr uint32_t kSlotBytes = kWave * CHUNK;          // one slot for every lane
    static constexpr uint32_t kInRing = SLOTS * kSlotBytes;
    static constexpr uint32_t kRow = ROUND * 8 + 16;               // output row stride (16-B aligned, staggered)
    static constexpr uint32_t kOutRing = kWave * kRow;
    static constexpr uint32_t kLanesPerRow = ROUND / 2;            // 16 B per lane in the store
    static constexpr uint32_t kRowsPerStep = kWave / kLanesPerRow;
    static constexpr uint32_t kSteps = kWave / kRowsPerStep;
    static constexpr uint32_t kBlock = WAVES * kWave;
    static_assert(CHUNK % 16 == 0 && (SLOTS & (SLOTS - 1)) == 0 && ROUND % 2 == 0, "cfg");
    __device__ static uint32_t swz(uint32_t l) { return (l >> 2) & (kPieces - 1); }
};

template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
__global__ __launch_bounds__(WAVES * 64) void decode_dma_kernel(const uint8_t* __restrict__ in,
                                                                const uint64_t* __restrict__ in_off,
                                                                const uint64_t* __restrict__ in_len,
                                                                uint32_t n, uint8_t* __restrict__ out,
                                                                const uint64_t* __restrict__ out_off,
                                                                const uint64_t* __restrict__ out_cap,
                                                                uint64_t* __restrict__ out_len,
                                                                int32_t* __restrict__ status) {
    using C = DmaCfg<CHUNK, SLOTS, ROUND, WAVES>;
    __shared__ __attribute__((aligned(16))) uint8_t in_all[WAVES * C::kInRing];
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[WAVES * C::kOutRing];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* iring = in_all + wave * C::kInRing;
    uint8_t* oring = ring_all + wave * C::kOutRing;
    const uint32_t unit = (blockIdx.x * WAVES + wave) * kWave + lane;
    const bool valid = unit < n;

    const uint8_t* src = in;
    uint64_t P = 0, capw = 0;
    uint8_t* dstb = out;
    int32_t st = ST_OK;
    if (valid) {
        src = in + in_off[unit];
        P = in_len[unit];
        dstb = out + out_off[unit];
        capw = out_cap[unit] >> 3;
        if (reinterpret_cast<uintptr_t>(dstb) & 7) st = ST_ARG;
        if (P > 0xFFFF0000ULL) st = ST_ARG;  // 32-bit stream offsets
    }
    bool live = valid && st == ST_OK;
    if (!live) P = 0;
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    const uint8_t* base = src - s;                    // 16-B aligned
    const uint32_t end = s + (uint32_t)P;             // logical stream [s, end)
    const uint32_t npieces = live ? (end + 15) >> 4 : 0;
    const uint32_t padded = npieces * 16;             // bytes the DMA ever delivers for this lane
    const uint32_t nchunks = (padded + CHUNK - 1) / CHUNK;
    uint32_t maxchunks = nchunks;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) maxchunks = max(maxchunks, (uint32_t)__shfl_xor((int)maxchunks, d, kWave));
    maxchunks = __builtin_amdgcn_readfirstlane(maxchunks);

    // DMA task descriptors: in pass k, lane L moves source piece kPieces*k + (i ^ swz(r))
    // of lane r = kTasks*g + L/kPieces into destination piece i = L % kPieces of r's slot k % SLOTS.
    uint64_t dsrc[C::kPieces];
    uint32_t dnp[C::kPieces], dpc[C::kPieces];
#pragma unroll
    for (uint32_t g = 0; g < C::kPieces; ++g) {
        const uint32_t r = C::kTasks * g + lane / C::kPieces;
        const uint32_t sp = (lane % C::kPieces) ^ C::swz(r);
        dsrc[g] = __shfl(reinterpret_cast<uint64_t>(base), r, kWave) + 16ULL * sp;
        dnp[g] = __shfl(npieces, r, kWave);
        dpc[g] = sp;
    }
    uint32_t issued = 0;  // wave-uniform: chunks issued for every lane
    auto dma_pass = [&]() {
        const uint32_t k = issued;
        uint8_t* slot = iring + (k & (SLOTS - 1)) * C::kSlotBytes;
#pragma unroll
        for (uint32_t g = 0; g < C::kPieces; ++g) {
            if (C::kPieces * k + dpc[g] < dnp[g]) {
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(dsrc[g] + (uint64_t)CHUNK * k),
                                                 (__attribute__((address_space(3))) void*)(slot + g * C::kTasks * CHUNK),
                                                 16, 0, 0);
            }
        }
        issued = k + 1;
    };

    uint32_t pos = s, lit = 0, pend_zero = 0, pend_lit = 0;
    uint64_t wo = 0;
    const uint32_t laneb = lane * CHUNK;
    const uint32_t swz16 = C::swz(lane) << 4;
    auto u64_at = [&](uint32_t y) -> uint64_t {  // y 8-aligned logical offset
        const uint32_t a = ((y / CHUNK) & (SLOTS - 1)) * C::kSlotBytes + laneb + ((y & (CHUNK - 1)) ^ swz16);
        return *reinterpret_cast<const uint64_t*>(iring + a);
    };
    // issue a pass while the slowest live lane has freed the slot the pass reuses
    auto may_issue = [&]() -> bool {
        const uint32_t mr = (pend_lit ? lit : pos) / CHUNK;  // oldest chunk still needed
        return issued < maxchunks && __all(!live || issued < mr + SLOTS);
    };

    for (uint32_t q = 0; q < SLOTS && may_issue(); ++q) dma_pass();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t landed = issued;

    uint64_t* myrow = reinterpret_cast<uint64_t*>(oring + lane * C::kRow);
    while (__any(live)) {
        const uint32_t limit = (landed * CHUNK >= padded) ? 0xFFFFFFFFu : landed * CHUNK;
        uint32_t nw = 0;
        bool frozen = false;
        for (uint32_t k = 0; k < ROUND; ++k) {
            const bool ok = live && !frozen;
            if (!__any(ok)) break;
            const bool isZ = pend_zero != 0;
            const bool isL = !isZ && pend_lit != 0;
            const bool isR = !isZ && !isL && pos < end;
            const uint32_t rp = isL ? lit : pos;
            const uint32_t y = rp & ~7u;
            const uint64_t a = u64_at(y), b = u64_at(y + 8);
            const uint32_t o = rp & 7;
            const uint32_t sh = 8 * o;
            const uint64_t lw = sh ? ((a >> sh) | (b << (64 - sh))) : a;         // literal word at rp
            const uint32_t t = (uint32_t)(a >> sh) & 0xFFu;                      // tag at rp
            const uint64_t pay = (o == 7) ? b : ((a >> (sh + 8)) | (b << (56 - sh)));  // bytes rp+1..rp+8
            uint32_t cnt = (uint32_t)(b >> (sh + 8)) & 0xFFu;                    // byte rp+9 (o <= 6)
            bool avail = y + 16 <= limit;
            const bool ff7 = ok && isR && avail && t == 0xFF && o == 7;
            if (__any(ff7)) {  // rare: FF count byte in the next 8-byte word
                if (ff7) {
                    avail = y + 24 <= limit;
                    if (avail) cnt = (uint32_t)u64_at(y + 16) & 0xFFu;
                }
            }
            const uint32_t kk = __popc(t);
            const bool tz = t == 0, tf = t == 0xFF;
            const uint32_t hdr = tz ? 2u : (tf ? 10u : 1u + kk);                  // bytes needed up front
            const uint32_t rlen = tf ? 10u + 8u * cnt : hdr;                      // record length
            const bool eof = (pos + hdr > end) || (pos + rlen > end);             // message.zig:152-191
            const bool stepZ = ok && isZ;
            const bool stepL = ok && isL && avail;
            const bool stepR = ok && isR && avail && !eof;
            const bool err = ok && isR && avail && eof;
            const bool fin = ok && !isZ && !isL && !isR;
            if (ok && (isL || isR) && !avail) frozen = true;
            if (err) st = ST_EOF;
            if (err || fin) live = false;
            const uint64_t rword = tz ? 0 : (tf ? pay : expand_word(pay, t));
            const uint64_t word = isZ ? 0 : (isL ? lw : rword);
            myrow[nw] = word;
            nw += (stepZ || stepL || stepR) ? 1u : 0u;
            pend_zero = stepZ ? pend_zero - 1 : ((stepR && tz) ? (uint32_t)pay & 0xFFu : pend_zero);
            pend_lit = stepL ? pend_lit - 1 : ((stepR && tf) ? cnt : pend_lit);
            lit = stepL ? lit + 8 : ((stepR && tf) ? pos + 10 : lit);
            pos = stepR ? pos + rlen : pos;
        }
        wave_lds_sync();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMAs issued at the last round end have landed
        landed = issued;
        // ---- cooperative store of this round's rows: lane L moves 16 B of one row ----------
        const uint64_t wo_round = wo;
#pragma unroll
        for (uint32_t j = 0; j < C::kSteps; ++j) {
            const uint32_t r = lane / C::kLanesPerRow + C::kRowsPerStep * j;
            const uint32_t i = lane % C::kLanesPerRow;
            const uint32_t rnw = __shfl(nw, r, kWave);
            const uint64_t rwo = __shfl(wo_round, r, kWave);
            const uint64_t rcap = __shfl(capw, r, kWave);
            uint8_t* rdst = reinterpret_cast<uint8_t*>(__shfl(reinterpret_cast<uint64_t>(dstb), r, kWave));
            const uint32_t w0 = 2 * i;
            if (w0 < rnw) {
                const uint8_t* rp = oring + r * C::kRow + 16 * i;
                const uint64_t g = rwo + w0;
                uint8_t* gp = rdst + 8 * g;
                const bool both = (w0 + 1 < rnw) && (g + 1 < rcap);
                if (g < rcap) {
                    if (both && !(reinterpret_cast<uintptr_t>(gp) & 15)) {
                        *reinterpret_cast<uint4*>(gp) = *reinterpret_cast<const uint4*>(rp);
                    } else {
                        *reinterpret_cast<uint64_t*>(gp) = *reinterpret_cast<const uint64_t*>(rp);
                        if (both) *reinterpret_cast<uint64_t*>(gp + 8) = *reinterpret_cast<const uint64_t*>(rp + 8);
                    }
                }
            }
        }
        wo += nw;
        for (uint32_t q = 0; q < 2 && may_issue(); ++q) dma_pass();
        wave_lds_sync();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the wave exits
    if (!valid) return;
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    out_len[unit] = 8 * wo;
    status[unit] = (wo > capw) ? ST_SPACE : ST_OK;
}

// Two-phase round: (1) WALK — the only serial part: per output word, follow the
// record chain using tag/count bytes only (ds_read_u8), and record the word's
// kind and source position in static registers; (2) EXPAND — ROUND independent
// words (unrolled), each reading its 16-byte window and expanding it, written to
// static ring offsets. The walk is ~15 instructions per record; the expansion's
// LDS latency is hidden by ILP across the round's words.
template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
__global__ __launch_bounds__(WAVES * 64) void decode_walk_kernel(const uint8_t* __restrict__ in,
                                                                 const uint64_t* __restrict__ in_off,
                                                                 const uint64_t* __restrict__ in_len,
                                                                 uint32_t n, uint8_t* __restrict__ out,
                                                                 const uint64_t* __restrict__ out_off,
                                                                 const uint64_t* __restrict__ out_cap,
                                                                 uint64_t* __restrict__ out_len,
                                                                 int32_t* __restrict__ status) {
    using C = DmaCfg<CHUNK, SLOTS, ROUND, WAVES>;
    __shared__ __attribute__((aligned(16))) uint8_t in_all[WAVES * C::kInRing];
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[WAVES * C::kOutRing];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* iring = in_all + wave * C::kInRing;
    uint8_t* oring = ring_all + wave * C::kOutRing;
    const uint32_t unit = (blockIdx.x * WAVES + wave) * kWave + lane;
    const bool valid = unit < n;

    const uint8_t* src = in;
    uint64_t P = 0, capw = 0;
    uint8_t* dstb = out;
    int32_t st = ST_OK;
    if (valid) {
        src = in + in_off[unit];
        P = in_len[unit];
        dstb = out + out_off[unit];
        capw = out_cap[unit] >> 3;
        if (reinterpret_cast<uintptr_t>(dstb) & 7) st = ST_ARG;
        if (P > 0x3FFF0000ULL) st = ST_ARG;  // 30-bit stream offsets
    }
    bool live = valid && st == ST_OK;
    if (!live) P = 0;
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    const uint8_t* base = src - s;
    const uint32_t end = s + (uint32_t)P;
    const uint32_t npieces = live ? (end + 15) >> 4 : 0;
    const uint32_t padded = npieces * 16;
    const uint32_t nchunks = (padded + CHUNK - 1) / CHUNK;
    uint32_t maxchunks = nchunks;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) maxchunks = max(maxchunks, (uint32_t)__shfl_xor((int)maxchunks, d, kWave));
    maxchunks = __builtin_amdgcn_readfirstlane(maxchunks);

    uint64_t dsrc[C::kPieces];
    uint32_t dnp[C::kPieces], dpc[C::kPieces];
#pragma unroll
    for (uint32_t g = 0; g < C::kPieces; ++g) {
        const uint32_t r = C::kTasks * g + lane / C::kPieces;
        const uint32_t sp = (lane % C::kPieces) ^ C::swz(r);
        dsrc[g] = __shfl(reinterpret_cast<uint64_t>(base), r, kWave) + 16ULL * sp;
        dnp[g] = __shfl(npieces, r, kWave);
        dpc[g] = sp;
    }
    uint32_t issued = 0;
    auto dma_pass = [&]() {
        const uint32_t k = issued;
        uint8_t* slot = iring + (k & (SLOTS - 1)) * C::kSlotBytes;
#pragma unroll
        for (uint32_t g = 0; g < C::kPieces; ++g) {
            if (C::kPieces * k + dpc[g] < dnp[g]) {
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(dsrc[g] + (uint64_t)CHUNK * k),
                                                 (__attribute__((address_space(3))) void*)(slot + g * C::kTasks * CHUNK),
                                                 16, 0, 0);
            }
        }
        issued = k + 1;
    };

    uint32_t pos = s, lit = 0, pend_zero = 0, pend_lit = 0;
    uint64_t wo = 0;
    const uint32_t laneb = lane * CHUNK;
    const uint32_t swz16 = C::swz(lane) << 4;
    auto ring_addr = [&](uint32_t y) -> uint32_t {  // LDS offset of logical byte y
        return ((y / CHUNK) & (SLOTS - 1)) * C::kSlotBytes + laneb + ((y & (CHUNK - 1)) ^ swz16);
    };
    auto u8_at = [&](uint32_t y) -> uint32_t { return iring[ring_addr(y)]; };
    auto u64_at = [&](uint32_t y) -> uint64_t {  // y 8-aligned
        return *reinterpret_cast<const uint64_t*>(iring + ring_addr(y));
    };
    auto may_issue = [&]() -> bool {
        const uint32_t mr = (pend_lit ? lit : pos) / CHUNK;
        return issued < maxchunks && __all(!live || issued < mr + SLOTS);
    };

    for (uint32_t q = 0; q < SLOTS && may_issue(); ++q) dma_pass();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t landed = issued;

    uint8_t* myrow = oring + lane * C::kRow;
    while (__any(live)) {
        const uint32_t limit = (landed * CHUNK >= padded) ? 0xFFFFFFFFu : landed * CHUNK;
        // ---- WALK: kinds/positions of this round's words -------------------------------
        uint32_t srcpos[ROUND];
        uint32_t mixmask = 0, litmask = 0;  // bit k: word k is a mixed record / a literal word
        uint32_t nw = 0;
        bool frozen = false;
#pragma unroll
        for (uint32_t k = 0; k < ROUND; ++k) {
            const bool ok = live && !frozen;
            const bool isZ = pend_zero != 0;
            const bool isL = !isZ && pend_lit != 0;
            const bool isR = !isZ && !isL && pos < end;
            const uint32_t t = u8_at(pos);          // tag (meaningful when isR)
            const uint32_t c1 = u8_at(pos + 1);     // zero-run count
            const uint32_t c9 = u8_at(pos + 9);     // literal-run count
            const bool avail = isL ? ((lit & ~7u) + 16 <= limit) : (!isR || (pos & ~7u) + 24 <= limit);
            const bool go = ok && avail && (isZ || isL || isR);
            const bool tz = t == 0, tf = t == 0xFF;
            const uint32_t hdr = tz ? 2u : (tf ? 10u : 1u + __popc(t));
            const uint32_t rlen = tf ? 10u + 8u * c9 : hdr;
            const bool eof = isR && (pos + hdr > end || pos + rlen > end);  // message.zig:152-191
            const bool emit = go && !eof;
            if (ok && !avail) frozen = true;
            if (go && eof) { st = ST_EOF; live = false; }
            if (ok && !isZ && !isL && !isR) live = false;  // unit finished
            srcpos[k] = isL ? lit : (pos + (tf ? 1u : 0u));
            if (emit && isR && !tz && !tf) mixmask |= 1u << k;
            if (emit && (isL || (isR && tf))) litmask |= 1u << k;
            nw += emit ? 1u : 0u;
            const bool stepR = emit && isR;
            pend_zero = (emit && isZ) ? pend_zero - 1 : ((stepR && tz) ? c1 : pend_zero);
            const bool stepL = emit && isL;
            pend_lit = stepL ? pend_lit - 1 : ((stepR && tf) ? c9 : pend_lit);
            lit = stepL ? lit + 8 : ((stepR && tf) ? pos + 10 : lit);
            pos = stepR ? pos + rlen : pos;
        }
        // ---- EXPAND: independent words --------------------------------------------------
#pragma unroll
        for (uint32_t k = 0; k < ROUND; ++k) {
            uint64_t word = 0;
            if ((mixmask | litmask) & (1u << k)) {
                const uint32_t p = srcpos[k];
                const uint32_t y = p & ~7u;
                const uint64_t a = u64_at(y), b = u64_at(y + 8);
                const uint32_t o = p & 7;
                if (mixmask & (1u << k)) {
                    const uint32_t t = (uint32_t)(a >> (8 * o)) & 0xFFu;
                    const uint64_t pay = (o == 7) ? b : ((a >> (8 * o + 8)) | (b << (56 - 8 * o)));
                    word = expand_word(pay, t);
                } else {
                    word = o ? ((a >> (8 * o)) | (b << (64 - 8 * o))) : a;
                }
            }
            *reinterpret_cast<uint64_t*>(myrow + 8 * k) = word;
        }
        wave_lds_sync();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        landed = issued;
        const uint64_t wo_round = wo;
#pragma unroll
        for (uint32_t j = 0; j < C::kSteps; ++j) {
            const uint32_t r = lane / C::kLanesPerRow + C::kRowsPerStep * j;
            const uint32_t i = lane % C::kLanesPerRow;
            const uint32_t rnw = __shfl(nw, r, kWave);
            const uint64_t rwo = __shfl(wo_round, r, kWave);
            const uint64_t rcap = __shfl(capw, r, kWave);
            uint8_t* rdst = reinterpret_cast<uint8_t*>(__shfl(reinterpret_cast<uint64_t>(dstb), r, kWave));
            const uint32_t w0 = 2 * i;
            if (w0 < rnw) {
                const uint8_t* rp = oring + r * C::kRow + 16 * i;
                const uint64_t g = rwo + w0;
                uint8_t* gp = rdst + 8 * g;
                const bool both = (w0 + 1 < rnw) && (g + 1 < rcap);
                if (g < rcap) {
                    if (both && !(reinterpret_cast<uintptr_t>(gp) & 15)) {
                        *reinterpret_cast<uint4*>(gp) = *reinterpret_cast<const uint4*>(rp);
                    } else {
                        *reinterpret_cast<uint64_t*>(gp) = *reinterpret_cast<const uint64_t*>(rp);
                        if (both) *reinterpret_cast<uint64_t*>(gp + 8) = *reinterpret_cast<const uint64_t*>(rp + 8);
                    }
                }
            }
        }
        wo += nw;
        for (uint32_t q = 0; q < 2 && may_issue(); ++q) dma_pass();
        wave_lds_sync();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!valid) return;
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    out_len[unit] = 8 * wo;
    status[unit] = (wo > capw) ? ST_SPACE : ST_OK;
}

template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
static void launch_walk(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n, uint8_t* out,
                        const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                        hipStream_t stream) {
    constexpr uint32_t per = WAVES * kWave;
    decode_walk_kernel<CHUNK, SLOTS, ROUND, WAVES><<<(n + per - 1) / per, per, 0, stream>>>(
        in, in_off, in_len, n, out, out_off, out_cap, out_len, status);
}

// Register window fed from the LDS-DMA ring: the record step reads only
// registers (a 32-byte view q0..q3); the window advances 16 B at a time from the
// lane's ring with the next piece (nx0, nx1) read one advance ahead, so LDS
// latency stays off the record chain and global latency stays behind the DMA ring.
template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
__global__ __launch_bounds__(WAVES * 64) void decode_win_kernel(const uint8_t* __restrict__ in,
                                                                const uint64_t* __restrict__ in_off,
                                                                const uint64_t* __restrict__ in_len,
                                                                uint32_t n, uint8_t* __restrict__ out,
                                                                const uint64_t* __restrict__ out_off,
                                                                const uint64_t* __restrict__ out_cap,
                                                                uint64_t* __restrict__ out_len,
                                                                int32_t* __restrict__ status) {
    using C = DmaCfg<CHUNK, SLOTS, ROUND, WAVES>;
    __shared__ __attribute__((aligned(16))) uint8_t in_all[WAVES * C::kInRing];
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[WAVES * C::kOutRing];
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* iring = in_all + wave * C::kInRing;
    uint8_t* oring = ring_all + wave * C::kOutRing;
    const uint32_t unit = (blockIdx.x * WAVES + wave) * kWave + lane;
    const bool valid = unit < n;

    const uint8_t* src = in;
    uint64_t P = 0, capw = 0;
    uint8_t* dstb = out;
    int32_t st = ST_OK;
    if (valid) {
        src = in + in_off[unit];
        P = in_len[unit];
        dstb = out + out_off[unit];
        capw = out_cap[unit] >> 3;
        if (reinterpret_cast<uintptr_t>(dstb) & 7) st = ST_ARG;
        if (P > 0xFFFF0000ULL) st = ST_ARG;
    }
    bool live = valid && st == ST_OK;
    if (!live) P = 0;
    const uint32_t s = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
    const uint8_t* base = src - s;
    const uint32_t end = s + (uint32_t)P;
    const uint32_t npieces = live ? (end + 15) >> 4 : 0;
    const uint32_t padded = npieces * 16;
    const uint32_t nchunks = (padded + CHUNK - 1) / CHUNK;
    uint32_t maxchunks = nchunks;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) maxchunks = max(maxchunks, (uint32_t)__shfl_xor((int)maxchunks, d, kWave));
    maxchunks = __builtin_amdgcn_readfirstlane(maxchunks);

    uint64_t dsrc[C::kPieces];
    uint32_t dnp[C::kPieces], dpc[C::kPieces];
#pragma unroll
    for (uint32_t g = 0; g < C::kPieces; ++g) {
        const uint32_t r = C::kTasks * g + lane / C::kPieces;
        const uint32_t sp = (lane % C::kPieces) ^ C::swz(r);
        dsrc[g] = __shfl(reinterpret_cast<uint64_t>(base), r, kWave) + 16ULL * sp;
        dnp[g] = __shfl(npieces, r, kWave);
        dpc[g] = sp;
    }
    uint32_t issued = 0;
    auto dma_pass = [&]() {
        const uint32_t k = issued;
        uint8_t* slot = iring + (k & (SLOTS - 1)) * C::kSlotBytes;
#pragma unroll
        for (uint32_t g = 0; g < C::kPieces; ++g) {
            if (C::kPieces * k + dpc[g] < dnp[g]) {
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(dsrc[g] + (uint64_t)CHUNK * k),
                                                 (__attribute__((address_space(3))) void*)(slot + g * C::kTasks * CHUNK),
                                                 16, 0, 0);
            }
        }
        issued = k + 1;
    };
    const uint32_t laneb = lane * CHUNK;
    const uint32_t swzp = C::swz(lane);
    // 16-B piece q (logical piece index) of this lane, from the ring
    auto piece_at = [&](uint32_t q, uint64_t& lo, uint64_t& hi) {
        const uint32_t a = ((q / C::kPieces) & (SLOTS - 1)) * C::kSlotBytes + laneb + (((q % C::kPieces) ^ swzp) << 4);
        const uint4 v = *reinterpret_cast<const uint4*>(iring + a);
        lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
        hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
    };

    uint32_t pos = s, lit = 0, pend_zero = 0, pend_lit = 0;
    uint64_t wo = 0;
    uint32_t wb = 0;  // logical offset of q0 (piece wb/16); nx = piece wb/16 + 2
    uint64_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, nx0 = 0, nx1 = 0;
    auto may_issue = [&]() -> bool {
        const uint32_t mr = wb / CHUNK;  // the window's first piece is the oldest byte still needed
        return issued < maxchunks && __all(!live || issued < mr + SLOTS);
    };

    for (uint32_t q = 0; q < SLOTS && may_issue(); ++q) dma_pass();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t landed = issued;
    if (live) {
        piece_at(0, q0, q1);
        piece_at(1, q2, q3);
        piece_at(2, nx0, nx1);
    }

    uint64_t* myrow = reinterpret_cast<uint64_t*>(oring + lane * C::kRow);
    while (__any(live)) {
        const uint32_t limit = (landed * CHUNK >= padded) ? 0xFFFFFFFFu : landed * CHUNK;
        uint32_t nw = 0;
        for (uint32_t k = 0; k < ROUND; ++k) {
            if (!live) break;
            const uint32_t rp = pend_lit ? lit : pos;
            if (rp - wb >= 16) {  // advance the window by one piece (never more per word)
                if (wb + 64 > limit) break;  // piece wb/16 + 3 not landed yet: resume next round
                q0 = q2; q1 = q3; q2 = nx0; q3 = nx1;
                wb += 16;
                piece_at((wb >> 4) + 2, nx0, nx1);
            }
            const uint32_t o = rp - wb;  // < 16
            uint64_t word = 0;
            if (pend_zero) {
                --pend_zero;
            } else if (pend_lit) {
                word = view_word8(q0, q1, q2, q3, o);
                lit += 8;
                --pend_lit;
            } else if (pos < end) {
                const uint32_t t = view_byte(q0, q1, q2, q3, o);
                const uint64_t pay = view_word8(q0, q1, q2, q3, o + 1);
                if (t == 0x00) {  // message.zig:101-110
                    if (pos + 2 > end) { st = ST_EOF; live = false; break; }
                    pend_zero = (uint32_t)pay & 0xFFu;
                    pos += 2;
                } else if (t == 0xFF) {  // message.zig:112-128
                    const uint32_t c = view_byte(q0, q1, q2, q3, o + 9);
                    if (pos + 10 > end || pos + 10 + 8 * c > end) { st = ST_EOF; live = false; break; }
                    word = pay;
                    pend_lit = c;
                    lit = pos + 10;
                    pos += 10 + 8 * c;
                } else {  // message.zig:131-141
                    const uint32_t kk = __popc(t);
                    if (pos + 1 + kk > end) { st = ST_EOF; live = false; break; }
                    word = expand_word(pay, t);
                    pos += 1 + kk;
                }
            } else {
                live = false;  // unit finished
                break;
            }
            myrow[nw++] = word;
        }
        wave_lds_sync();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        landed = issued;
        const uint64_t wo_round = wo;
#pragma unroll
        for (uint32_t j = 0; j < C::kSteps; ++j) {
            const uint32_t r = lane / C::kLanesPerRow + C::kRowsPerStep * j;
            const uint32_t i = lane % C::kLanesPerRow;
            const uint32_t rnw = __shfl(nw, r, kWave);
            const uint64_t rwo = __shfl(wo_round, r, kWave);
            const uint64_t rcap = __shfl(capw, r, kWave);
            uint8_t* rdst = reinterpret_cast<uint8_t*>(__shfl(reinterpret_cast<uint64_t>(dstb), r, kWave));
            const uint32_t w0 = 2 * i;
            if (w0 < rnw) {
                const uint8_t* rpp = oring + r * C::kRow + 16 * i;
                const uint64_t g = rwo + w0;
                uint8_t* gp = rdst + 8 * g;
                const bool both = (w0 + 1 < rnw) && (g + 1 < rcap);
                if (g < rcap) {
                    if (both && !(reinterpret_cast<uintptr_t>(gp) & 15)) {
                        *reinterpret_cast<uint4*>(gp) = *reinterpret_cast<const uint4*>(rpp);
                    } else {
                        *reinterpret_cast<uint64_t*>(gp) = *reinterpret_cast<const uint64_t*>(rpp);
                        if (both) *reinterpret_cast<uint64_t*>(gp + 8) = *reinterpret_cast<const uint64_t*>(rpp + 8);
                    }
                }
            }
        }
        wo += nw;
        for (uint32_t q = 0; q < 2 && may_issue(); ++q) dma_pass();
        wave_lds_sync();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!valid) return;
    if (st != ST_OK) {
        out_len[unit] = 0;
        status[unit] = st;
        return;
    }
    out_len[unit] = 8 * wo;
    status[unit] = (wo > capw) ? ST_SPACE : ST_OK;
}

template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
static void launch_win(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n, uint8_t* out,
                       const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                       hipStream_t stream) {
    constexpr uint32_t per = WAVES * kWave;
    decode_win_kernel<CHUNK, SLOTS, ROUND, WAVES><<<(n + per - 1) / per, per, 0, stream>>>(
        in, in_off, in_len, n, out, out_off, out_cap, out_len, status);
}

template <uint32_t CHUNK, uint32_t SLOTS, uint32_t ROUND, uint32_t WAVES>
static void launch_dma(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n, uint8_t* out,
                       const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                       hipStream_t stream) {
    constexpr uint32_t per = WAVES * kWave;
    decode_dma_kernel<CHUNK, SLOTS, ROUND, WAVES><<<(n + per - 1) / per, per, 0, stream>>>(
        in, in_off, in_len, n, out, out_off, out_cap, out_len, status);
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

hipError_t launch_encode(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                         int32_t* status, bool write, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (write)
        encode_kernel<true><<<blocks_for(n), kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                   out_len, status);
    else
        encode_kernel<false><<<blocks_for(n), kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                    out_len, status);
    return hipGetLastError();
}

static int decode_variant() {
    static int v = [] {
        const char* e = getenv("CPK_DECODE_VARIANT");  // experiment switch; default 2
        return e ? atoi(e) : 2;
    }();
    return v;
}

hipError_t launch_decode(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                         int32_t* status, bool write, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (write) {
        switch (decode_variant()) {
            case 1: launch_dma<64, 4, 16, 2>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 3: launch_dma<32, 4, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 4: launch_dma<32, 4, 8, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 5: launch_dma<64, 2, 8, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 6: launch_dma<32, 2, 8, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 7: launch_dma<64, 4, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 12: launch_win<64, 4, 16, 2>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 13: launch_win<32, 4, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 14: launch_win<32, 4, 8, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 15: launch_win<64, 2, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 16: launch_win<64, 4, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 8: launch_walk<64, 4, 16, 2>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 9: launch_walk<64, 4, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 10: launch_walk<32, 4, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            case 11: launch_walk<64, 2, 16, 1>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status, stream);
                    return hipGetLastError();
            default: break;
        }
    }
    if (write && (decode_variant() == 2 || (decode_variant() >= 20 && decode_variant() <= 23))) {
        const uint32_t blocks = (n + kStreamBlock - 1) / kStreamBlock;
        switch (decode_variant()) {
            case 20: decode_stream_kernel<256><<<blocks, kStreamBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status); break;
            case 21: decode_stream_kernel<512><<<blocks, kStreamBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status); break;
            case 22: decode_stream_kernel<1024><<<blocks, kStreamBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status); break;
            case 23: decode_stream_kernel<128><<<blocks, kStreamBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status); break;
            default: decode_stream_kernel<0><<<blocks, kStreamBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap, out_len, status); break;
        }
        return hipGetLastError();
    }
    if (decode_variant() >= 1) {
        const uint32_t blocks = (n + kBlock - 1) / kBlock;
        if (write)
            decode_lane_kernel<true><<<blocks, kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                     out_len, status);
        else
            decode_lane_kernel<false><<<blocks, kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                      out_len, status);
        return hipGetLastError();
    }
    if (write)
        decode_kernel<true><<<blocks_for(n), kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                   out_len, status);
    else
        decode_kernel<false><<<blocks_for(n), kBlock, 0, stream>>>(in, in_off, in_len, n, out, out_off, out_cap,
                                                                    out_len, status);
    return hipGetLastError();
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
