// capnp_packed_abi.cpp — the C-ABI boundary (include/capnp_packed.h).
//
// Conventions follow the reference's only FFI, src/wasm/capnp_host_abi.zig:
// integer status codes, a last-error message (:165-184), and a version query
// (:60-70). Single-buffer calls run ONE unit through the GPU via a small
// mutex-guarded device context; batch calls only enqueue kernels on the
// caller's stream. There is no CPU code path: without a gfx950 device every
// compute entry point returns CAPNP_PACKED_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "capnp_packed.h"
#include "kernels.h"

namespace {

thread_local std::string g_last_error;

int fail(int status, const std::string& msg) {
    g_last_error = msg;
    return status;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(CAPNP_PACKED_DEVICE_ERROR, std::string(what) + ": " + hipGetErrorString(e));
}

std::once_flag g_init_once;
int g_init_status = CAPNP_PACKED_NO_DEVICE;
std::string g_init_error;

void device_init() {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        g_init_status = CAPNP_PACKED_NO_DEVICE;
        g_init_error = "no HIP device visible";
        return;
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) {
        g_init_status = CAPNP_PACKED_DEVICE_ERROR;
        g_init_error = std::string("hipGetDeviceProperties: ") + hipGetErrorString(e);
        return;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_init_status = CAPNP_PACKED_NO_DEVICE;
        g_init_error = std::string("device is ") + prop.gcnArchName + ", this library is built for gfx950 only";
        return;
    }
    g_init_status = CAPNP_PACKED_OK;
}

int ensure_device() {
    std::call_once(g_init_once, device_init);
    if (g_init_status != CAPNP_PACKED_OK) return fail(g_init_status, g_init_error);
    return CAPNP_PACKED_OK;
}

// Device context for the single-buffer host entry points: grow-only device buffers and
// pinned host staging (the caller's pageable bytes are copied into pinned memory, so the
// H2D / D2H copies run as DMA at full PCIe rate), one stream, the meta block's host copy
// in pinned memory too.
struct HostCtx {
    std::mutex mu;
    hipStream_t stream = nullptr;
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* d_out = nullptr;
    size_t out_cap = 0;
    uint8_t* h_in = nullptr;  // pinned staging
    size_t h_in_cap = 0;
    uint8_t* h_out = nullptr;
    size_t h_out_cap = 0;
    uint64_t* d_meta = nullptr;  // in_off, in_len, out_off, out_cap, out_len, status (as u64), consumed
    uint64_t* h_meta = nullptr;

    int init() {
        if (stream) return CAPNP_PACKED_OK;
        hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
        e = hipMalloc(&d_meta, 8 * sizeof(uint64_t));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(meta)");
        e = hipHostMalloc(reinterpret_cast<void**>(&h_meta), 8 * sizeof(uint64_t), hipHostMallocDefault);
        if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(meta)");
        return CAPNP_PACKED_OK;
    }
    static size_t grow(size_t need) { return need < 65536 ? 65536 : need + need / 2; }
    // A buffer grown by an unusually large call is given back on the next call that needs a
    // quarter of it or less (above 64 MiB): the context does not pin its peak for the process.
    static bool keep(size_t need, size_t cap) { return need <= cap && !(cap > (64u << 20) && need <= cap / 4); }
    int reserve(uint8_t** p, size_t* cap, size_t need) {
        if (*p && keep(need, *cap)) return CAPNP_PACKED_OK;
        if (need > (SIZE_MAX / 3) * 2) return fail(CAPNP_PACKED_OUT_OF_SPACE, "workspace size overflows size_t");
        const size_t want = grow(need);
        if (*p) (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
        hipError_t e = hipMalloc(p, want);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
        *cap = want;
        return CAPNP_PACKED_OK;
    }
    int reserve_host(uint8_t** p, size_t* cap, size_t need) {
        if (*p && keep(need, *cap)) return CAPNP_PACKED_OK;
        if (need > (SIZE_MAX / 3) * 2) return fail(CAPNP_PACKED_OUT_OF_SPACE, "staging size overflows size_t");
        const size_t want = grow(need);
        if (*p) (void)hipHostFree(*p);
        *p = nullptr;
        *cap = 0;
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(p), want, hipHostMallocDefault);
        if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(staging)");
        *cap = want;
        return CAPNP_PACKED_OK;
    }
};

HostCtx g_ctx;

// Device buffers of capnp_packed_frame_connections (grow-only; its own streams and lock,
// so framing never waits on a single-buffer call). Frame slots are double-buffered: round r
// decodes into d_out[r % 2] while the copy stream moves round r - 1's frames to the host.
struct FrameCtx {
    std::mutex mu;
    hipStream_t stream = nullptr;
    hipStream_t copy = nullptr;   // frames D2H, overlapping the next round
    hipEvent_t ev_done[2] = {nullptr, nullptr};  // round into d_out[b] decoded
    hipEvent_t ev_copied[2] = {nullptr, nullptr};  // frames of d_out[b] on the host
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* d_out[2] = {nullptr, nullptr};
    size_t out_cap[2] = {0, 0};
    uint8_t* d_meta = nullptr;
    size_t meta_cap = 0;

    int init() {
        if (stream) return CAPNP_PACKED_OK;
        hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&copy, hipStreamNonBlocking);
        for (int b = 0; b < 2 && e == hipSuccess; ++b) {
            e = hipEventCreateWithFlags(&ev_done[b], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev_copied[b], hipEventDisableTiming);
        }
        return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "hipStreamCreate(framer)");
    }
    int reserve(uint8_t** p, size_t* cap, size_t need) {
        if (need <= *cap && *p) return CAPNP_PACKED_OK;
        if (need > (SIZE_MAX / 3) * 2) return fail(CAPNP_PACKED_OUT_OF_SPACE, "workspace size overflows size_t");
        const size_t want = need < 65536 ? 65536 : need + need / 2;
        if (*p) (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(p), want);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(framer)");
        *cap = want;
        return CAPNP_PACKED_OK;
    }
};

FrameCtx g_fr;

// Largest unpacked size of n packed bytes: a 2-byte zero-run record expands to 256 words.
uint64_t unpack_bound(size_t n) { return n > (UINT64_MAX / 1024) ? UINT64_MAX : 1024ull * n; }

// Run one unit through a batch kernel. kind: 0 encode, 1 decode, 2 decoded size, 3 encoded size,
// 4 read message (reader.zig:84-156; *used_out = packed bytes consumed). The input crosses
// PCIe once (pinned staging), the kernels run with an output slot of `slot` bytes, and the
// output comes back only when the unit is OK; *len_out is out_len (for OUT_OF_SPACE: the
// size the unit needs).
// reuse_in: the device already holds `in` from the previous call (a retry with a larger slot).
// Single units up to these sizes take one kernel (cpk::launch_decode_one / launch_encode_one);
// DESIGN.md §6.1 has the measured crossover.
constexpr size_t kFastDecodeMax = 24 * 1024;  // packed bytes (the serial window walk passes the batch path near 32 KB)
constexpr size_t kFastEncodeMax = 4096;       // unpacked bytes: one 512-word tile

int run_single(int kind, const uint8_t* in, size_t n, uint8_t* out, size_t slot, uint64_t* len_out,
               uint64_t* used_out = nullptr, bool reuse_in = false) {
    int st = g_ctx.init();
    if (st) return st;
    if (n > SIZE_MAX - 16 || slot > SIZE_MAX - 16) return fail(CAPNP_PACKED_OUT_OF_SPACE, "buffer size overflows size_t");
    if (!reuse_in) {
        if ((st = g_ctx.reserve(&g_ctx.d_in, &g_ctx.in_cap, n + 16))) return st;
        if ((st = g_ctx.reserve_host(&g_ctx.h_in, &g_ctx.h_in_cap, n + 16))) return st;
    }
    const bool write = (kind == 0 || kind == 1 || kind == 4);
    if (write && (st = g_ctx.reserve(&g_ctx.d_out, &g_ctx.out_cap, slot + 16))) return st;
    uint64_t* const hm = g_ctx.h_meta;
    // one kernel for a single unit the one-unit kernels take (kFastDecodeMax / kFastEncodeMax)
    const bool one = n > 0 && ((kind == 1 && n <= kFastDecodeMax) || ((kind == 0 || kind == 3) && n <= kFastEncodeMax));
    uint64_t meta[7] = {0, n, 0, slot, 0, 0, 0};  // in_off, in_len, out_off, out_cap, out_len, status, consumed
    if (one && kind == 1) {
        const int32_t need = cpk::decode_one_status();  // decode_wave_kernel<kWvMarked> takes marked units
        std::memcpy(&meta[5], &need, sizeof(need));
    }
    std::memcpy(hm, meta, sizeof(meta));
    hipStream_t s = g_ctx.stream;
    hipError_t e = hipSuccess;
    if (n && !reuse_in) {
        std::memcpy(g_ctx.h_in, in, n);
        e = hipMemcpyAsync(g_ctx.d_in, g_ctx.h_in, n, hipMemcpyHostToDevice, s);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(g_ctx.d_meta, hm, sizeof(meta), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(H2D)");
    uint64_t* m = g_ctx.d_meta;
    int32_t* d_status = reinterpret_cast<int32_t*>(m + 5);
    if (one && kind == 1)
        e = cpk::launch_decode_one(g_ctx.d_in, m, m + 1, g_ctx.d_out, m + 2, m + 3, m + 4, d_status, s);
    else if (one)
        e = cpk::launch_encode_one(g_ctx.d_in, m, m + 1, g_ctx.d_out, m + 2, m + 3, m + 4, d_status, write, s);
    else if (kind == 0 || kind == 3)
        e = cpk::launch_encode(g_ctx.d_in, m, m + 1, 1, g_ctx.d_out, m + 2, m + 3, m + 4, d_status, write, nullptr, 0,
                               s);
    else if (kind == 4)
        e = cpk::launch_read_message(g_ctx.d_in, m, m + 1, 1, g_ctx.d_out, m + 2, m + 3, m + 4, m + 6, d_status, s);
    else
        e = cpk::launch_decode(g_ctx.d_in, m, m + 1, 1, g_ctx.d_out, m + 2, m + 3, m + 4, d_status, write, nullptr, 0,
                               s);
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    e = hipMemcpyAsync(hm, g_ctx.d_meta, sizeof(meta), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(D2H)");
    int32_t status;
    std::memcpy(&status, &hm[5], sizeof(status));
    *len_out = hm[4];
    if (used_out) *used_out = hm[6];
    if (status == CAPNP_PACKED_OK && write && hm[4]) {
        const size_t len = (size_t)hm[4];
        if ((st = g_ctx.reserve_host(&g_ctx.h_out, &g_ctx.h_out_cap, len))) return st;
        e = hipMemcpyAsync(g_ctx.h_out, g_ctx.d_out, len, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy(D2H out)");
        std::memcpy(out, g_ctx.h_out, len);
    }
    if (status != CAPNP_PACKED_OK) g_last_error = capnp_packed_status_name(status);
    return status;
}

int check_batch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, uint32_t n,
                const uint64_t* d_len, const int32_t* d_status) {
    if (n == 0) return CAPNP_PACKED_OK;
    if (!d_in_off || !d_in_len || !d_len || !d_status) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null batch pointer");
    (void)d_in;
    return ensure_device();
}

}  // namespace

extern "C" {

uint32_t capnp_packed_abi_version(void) { return CAPNP_PACKED_ABI_VERSION; }

const char* capnp_packed_last_error(void) { return g_last_error.c_str(); }

const char* capnp_packed_status_name(int status) {
    switch (status) {
        case CAPNP_PACKED_OK: return "Ok";
        case CAPNP_PACKED_INVALID_MESSAGE_SIZE: return "InvalidMessageSize";
        case CAPNP_PACKED_UNEXPECTED_EOF: return "UnexpectedEof";
        case CAPNP_PACKED_OVERFLOW: return "Overflow";
        case CAPNP_PACKED_OUT_OF_SPACE: return "OutOfSpace";
        case CAPNP_PACKED_INVALID_ARGUMENT: return "InvalidArgument";
        case CAPNP_PACKED_DEVICE_ERROR: return "DeviceError";
        case CAPNP_PACKED_NO_DEVICE: return "NoDevice";
        case CAPNP_PACKED_END_OF_STREAM: return "EndOfStream";
        case CAPNP_PACKED_INVALID_SEGMENT_COUNT: return "InvalidSegmentCount";
        case CAPNP_PACKED_SEGMENT_COUNT_LIMIT_EXCEEDED: return "SegmentCountLimitExceeded";
        case CAPNP_PACKED_MESSAGE_TOO_LARGE: return "MessageTooLarge";
        case CAPNP_PACKED_INVALID_PACKED_MESSAGE: return "InvalidPackedMessage";
        case CAPNP_PACKED_TRUNCATED_MESSAGE: return "TruncatedMessage";
        case CAPNP_PACKED_EMPTY_MESSAGE: return "EmptyMessage";
        case CAPNP_PACKED_NESTING_LIMIT_EXCEEDED: return "NestingLimitExceeded";
        case CAPNP_PACKED_INVALID_SEGMENT_ID: return "InvalidSegmentId";
        case CAPNP_PACKED_INVALID_POINTER: return "InvalidPointer";
        case CAPNP_PACKED_OUT_OF_BOUNDS: return "OutOfBounds";
        case CAPNP_PACKED_TRAVERSAL_LIMIT_EXCEEDED: return "TraversalLimitExceeded";
        case CAPNP_PACKED_INVALID_FAR_POINTER: return "InvalidFarPointer";
        case CAPNP_PACKED_INVALID_INLINE_COMPOSITE_POINTER: return "InvalidInlineCompositePointer";
        case CAPNP_PACKED_LIST_TOO_LARGE: return "ListTooLarge";
        default: return "Unknown";
    }
}

size_t capnp_packed_encode_bound(size_t n) { return 10 * (n / 8); }

int capnp_packed_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    if (!out_len) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "out_len is null");
    *out_len = 0;
    if ((n && !in) || (cap && !out)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null buffer");
    if (n % 8) return fail(CAPNP_PACKED_INVALID_MESSAGE_SIZE, "InvalidMessageSize");  // message.zig:201
    int st = ensure_device();
    if (st) return st;
    std::lock_guard<std::mutex> lock(g_ctx.mu);
    size_t bound = capnp_packed_encode_bound(n);
    uint64_t len = 0;
    st = run_single(0, in, n, out, cap < bound ? cap : bound, &len);
    *out_len = (size_t)len;
    return st;
}

int capnp_packed_decoded_size(const uint8_t* in, size_t n, size_t* out_size) {
    if (!out_size) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "out_size is null");
    *out_size = 0;
    if (n && !in) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null buffer");
    int st = ensure_device();
    if (st) return st;
    std::lock_guard<std::mutex> lock(g_ctx.mu);
    uint64_t len = 0;
    st = run_single(2, in, n, nullptr, 0, &len);
    if (st == CAPNP_PACKED_OK) *out_size = (size_t)len;
    return st;
}

int capnp_packed_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    if (!out_len) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "out_len is null");
    *out_len = 0;
    if ((n && !in) || (cap && !out)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null buffer");
    int st = ensure_device();
    if (st) return st;
    std::lock_guard<std::mutex> lock(g_ctx.mu);
    // One H2D and one decode into a device slot of min(cap, 8 n, at least 64 KiB) bytes: dense
    // data expands ~1.1-2x, so that slot nearly always holds it, and a large reusable caller
    // buffer does not size the device slot (up to 1024 n). A unit that does not fit ends
    // OUT_OF_SPACE with its size in out_len (the output is copied back only when OK, so the
    // caller's buffer is untouched, message.zig:90); if the caller's capacity holds that size
    // the decode runs again from the input already on the device, into a slot of that size.
    const uint64_t bound = unpack_bound(n);
    const uint64_t room = cap < bound ? cap : bound;
    const uint64_t guess = n > (UINT64_MAX / 8) ? UINT64_MAX : (8ull * n < 65536 ? 65536 : 8ull * n);
    const uint64_t first = room < guess ? room : guess;
    uint64_t len = 0;
    st = run_single(1, in, n, out, (size_t)first, &len);
    if (st == CAPNP_PACKED_OUT_OF_SPACE && first < room && len <= room)
        st = run_single(1, in, n, out, (size_t)len, &len, nullptr, true);
    *out_len = (st == CAPNP_PACKED_OK || st == CAPNP_PACKED_OUT_OF_SPACE) ? (size_t)len : 0;
    return st;
}

size_t capnp_packed_batch_workspace_bytes(uint32_t n) { return cpk::queue_bytes(n); }

int capnp_packed_set_decoder(int decoder) {
    if (decoder < CAPNP_PACKED_DECODER_AUTO || decoder > CAPNP_PACKED_DECODER_WORDS)
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "unknown decoder");
    if (!cpk::decoder_built(decoder))
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "decoder removed from the library (round 5; DESIGN.md §2.3a, §2.3b)");
    return cpk::set_decoder(decoder);
}

int capnp_packed_set_all_or_nothing(int on) { return cpk::set_all_or_nothing(on); }

uint32_t capnp_packed_set_launch_flags(uint32_t flags) {
    return cpk::set_launch_flags(flags & (CAPNP_PACKED_LAUNCH_LONG_INLINE | CAPNP_PACKED_LAUNCH_MID_SIDE_STREAM |
                                          CAPNP_PACKED_LAUNCH_CLASS_SCAN));
}

int capnp_packed_stream_release(void* stream) {
    int st = ensure_device();
    if (st) return st;
    hipError_t e = cpk::release_stream(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "stream release");
}

int capnp_packed_stream_queue_info(void* stream, size_t* bytes, uint32_t* kept) {
    if (!bytes || !kept) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null output");
    *bytes = 0;
    *kept = 0;
    int st = ensure_device();
    if (st) return st;
    cpk::stream_queue_info(static_cast<hipStream_t>(stream), bytes, kept);
    return CAPNP_PACKED_OK;
}

int capnp_packed_stream_contexts(uint32_t* count) {
    if (!count) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null output");
    *count = 0;
    int st = ensure_device();
    if (st) return st;
    *count = cpk::stream_context_count();
    return CAPNP_PACKED_OK;
}

// The kernels address the workspace as u32 counters, 16-B table entries and 64-B
// record stores at 256-B offsets: it must be 256-B aligned (hipMalloc's alignment).
static int check_ws(const void* ws, size_t bytes, uint32_t n) {
    if (!ws) return CAPNP_PACKED_OK;
    if (reinterpret_cast<uintptr_t>(ws) & 255)
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "workspace not 256-B aligned");
    if (bytes < cpk::queue_bytes(n))
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "workspace smaller than capnp_packed_batch_workspace_bytes(n)");
    return CAPNP_PACKED_OK;
}

int capnp_packed_encode_batch_ws(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                 uint32_t n, uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_cap,
                                 uint64_t* d_out_len, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                                 void* stream) {
    int st = check_batch(d_in, d_in_off, d_in_len, n, d_out_len, d_status);
    if (st || n == 0) return st;
    if (!d_out_off || !d_out_cap) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null output slot arrays");
    if ((st = check_ws(d_workspace, workspace_bytes, n))) return st;
    hipError_t e = cpk::launch_encode(d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len,
                                      d_status, true, d_workspace, workspace_bytes, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "encode launch");
}

int capnp_packed_encode_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                              uint32_t n, uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_cap,
                              uint64_t* d_out_len, int32_t* d_status, void* stream) {
    return capnp_packed_encode_batch_ws(d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len,
                                        d_status, nullptr, 0, stream);
}

int capnp_packed_encoded_size_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint64_t* d_out_len, int32_t* d_status, void* stream) {
    int st = check_batch(d_in, d_in_off, d_in_len, n, d_out_len, d_status);
    if (st || n == 0) return st;
    hipError_t e = cpk::launch_encode(d_in, d_in_off, d_in_len, n, nullptr, nullptr, nullptr, d_out_len, d_status,
                                      false, nullptr, 0, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "encode-size launch");
}

int capnp_packed_decode_batch_ws(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                 uint32_t n, uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_cap,
                                 uint64_t* d_out_len, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                                 void* stream) {
    int st = check_batch(d_in, d_in_off, d_in_len, n, d_out_len, d_status);
    if (st || n == 0) return st;
    if (!d_out_off || !d_out_cap) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null output slot arrays");
    if ((st = check_ws(d_workspace, workspace_bytes, n))) return st;
    hipError_t e = cpk::launch_decode(d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len,
                                      d_status, true, d_workspace, workspace_bytes, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "decode launch");
}

int capnp_packed_decode_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                              uint32_t n, uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_cap,
                              uint64_t* d_out_len, int32_t* d_status, void* stream) {
    return capnp_packed_decode_batch_ws(d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len,
                                        d_status, nullptr, 0, stream);
}

int capnp_packed_decoded_size_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint64_t* d_out_len, int32_t* d_status, void* stream) {
    int st = check_batch(d_in, d_in_off, d_in_len, n, d_out_len, d_status);
    if (st || n == 0) return st;
    hipError_t e = cpk::launch_decode(d_in, d_in_off, d_in_len, n, nullptr, nullptr, nullptr, d_out_len, d_status,
                                      false, nullptr, 0, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "decode-size launch");
}

int capnp_packed_read_message_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint8_t* d_out, const uint64_t* d_out_off,
                                    const uint64_t* d_out_cap, uint64_t* d_out_len, uint64_t* d_consumed,
                                    int32_t* d_status, void* stream) {
    int st = check_batch(d_in, d_in_off, d_in_len, n, d_out_len, d_status);
    if (st || n == 0) return st;
    if (!d_out_off || !d_out_cap || !d_consumed) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null output arrays");
    hipError_t e = cpk::launch_read_message(d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len,
                                            d_consumed, d_status, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "read-message launch");
}

int capnp_packed_read_message(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len,
                              size_t* consumed) {
    if (!out_len || !consumed) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "out_len/consumed is null");
    *out_len = 0;
    *consumed = 0;
    if ((n && !in) || (cap && !out)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null buffer");
    int st = ensure_device();
    if (st) return st;
    std::lock_guard<std::mutex> lock(g_ctx.mu);
    // reader.zig can produce at most a 512-segment header (257 words) plus
    // max_total_words (8 Mi, reader.zig:6) words: a larger cap is clamped, so the
    // device slot is sized by what the reader can write, not by the caller's buffer
    const size_t kMaxFramed = (257ull + 8ull * 1024 * 1024) * 8;
    uint64_t len = 0, used = 0;
    st = run_single(4, in, n, out, cap < kMaxFramed ? cap : kMaxFramed, &len, &used);
    *out_len = (size_t)len;
    *consumed = (size_t)used;
    return st;
}

int capnp_packed_encode_message_batch(const uint64_t* d_seg_ptr, const uint64_t* d_seg_len,
                                      const uint32_t* d_seg_first, const uint32_t* d_seg_count, uint32_t n,
                                      uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_cap,
                                      uint64_t* d_out_len, int32_t* d_status, void* stream) {
    if (n == 0) return CAPNP_PACKED_OK;
    if (!d_seg_first || !d_seg_count || !d_out_len || !d_status)
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null batch pointer");
    const bool write = d_out != nullptr;
    if (write && (!d_out_off || !d_out_cap)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null output slot arrays");
    int st = ensure_device();
    if (st) return st;
    hipError_t e = cpk::launch_encode_message(d_seg_ptr, d_seg_len, d_seg_first, d_seg_count, n, d_out, d_out_off,
                                              d_out_cap, d_out_len, d_status, write, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "encode-message launch");
}

int capnp_packed_message_init_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint32_t max_segs, uint32_t* d_seg_count, uint64_t* d_seg_off,
                                    uint64_t* d_seg_len, int32_t* d_status, void* stream) {
    if (n == 0) return CAPNP_PACKED_OK;
    if (!d_in_off || !d_in_len || !d_seg_count || !d_status || (max_segs && (!d_seg_off || !d_seg_len)))
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null batch pointer");
    int st = ensure_device();
    if (st) return st;
    hipError_t e = cpk::launch_message_init(d_in, d_in_off, d_in_len, n, max_segs, d_seg_count, d_seg_off, d_seg_len,
                                            d_status, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "message-init launch");
}

int capnp_packed_validate_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                uint32_t n, uint64_t segment_count_limit, uint64_t traversal_limit_words,
                                uint32_t nesting_limit, int32_t* d_status, uint64_t* d_words, void* stream) {
    if (n == 0) return CAPNP_PACKED_OK;
    if (!d_in_off || !d_in_len || !d_status) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null batch pointer");
    int st = ensure_device();
    if (st) return st;
    hipError_t e = cpk::launch_validate(d_in, d_in_off, d_in_len, n, segment_count_limit, traversal_limit_words,
                                        nesting_limit, d_status, d_words, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "validate launch");
}

size_t capnp_packed_scan_scratch_bytes(uint32_t n) { return cpk::scan_scratch_bytes(n); }

int capnp_packed_lengths_to_offsets(const uint64_t* d_len, uint32_t n, uint64_t base, uint64_t* d_off,
                                    void* d_scratch, size_t scratch_bytes, void* stream) {
    if (!d_off || !d_scratch || (n && !d_len)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null pointer");
    if (scratch_bytes < cpk::scan_scratch_bytes(n)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "scratch too small");
    int st = ensure_device();
    if (st) return st;
    hipError_t e = cpk::launch_scan(d_len, n, base, d_off, static_cast<uint64_t*>(d_scratch),
                                    static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "scan launch");
}

int capnp_packed_generate(uint8_t* d_out, uint64_t n_units, uint64_t unit_bytes, uint64_t unit_base,
                          uint64_t seed, uint32_t zero_thresh, void* stream) {
    if (!d_out && n_units) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null d_out");
    if (unit_bytes % 8) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "unit_bytes % 8 != 0");
    int st = ensure_device();
    if (st) return st;
    hipError_t e = cpk::launch_generate(d_out, n_units, unit_bytes, unit_base, seed, zero_thresh,
                                        static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "generate launch");
}

int capnp_packed_frame_connections(const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                                   const uint64_t* in_len, uint32_t n, uint64_t* slot_guess, uint8_t* frames,
                                   uint64_t frames_cap, uint64_t* frame_off, uint64_t* frame_len,
                                   uint32_t* frame_conn, uint32_t max_frames, uint64_t* consumed, int32_t* status,
                                   uint32_t* n_frames) {
    if (!n_frames) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "n_frames is null");
    *n_frames = 0;
    if (n == 0) return CAPNP_PACKED_OK;
    if (!in_off || !in_len || !slot_guess || !consumed || !status || (in_bytes && !in) ||
        (max_frames && (!frame_off || !frame_len || !frame_conn)) || (frames_cap && !frames))
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null pointer");
    for (uint32_t c = 0; c < n; ++c)
        if (in_off[c] > in_bytes || in_len[c] > in_bytes - in_off[c])
            return fail(CAPNP_PACKED_INVALID_ARGUMENT, "connection bytes outside the input buffer");
    int st = ensure_device();
    if (st) return st;
    std::lock_guard<std::mutex> lock(g_fr.mu);
    if ((st = g_fr.init())) return st;
    // no copy of an earlier call may still write into its caller's frames buffer: each call
    // ends with the copy stream drained (copies_done below), also on its error paths
    struct CopiesDone {
        ~CopiesDone() { (void)hipStreamSynchronize(g_fr.copy); }
    } copies_done;
    if ((st = g_fr.reserve(&g_fr.d_in, &g_fr.in_cap, in_bytes + 16))) return st;
    if ((st = g_fr.reserve(&g_fr.d_meta, &g_fr.meta_cap, (size_t)n * 7 * sizeof(uint64_t)))) return st;
    const hipStream_t s = g_fr.stream;
    hipError_t e = in_bytes ? hipMemcpyAsync(g_fr.d_in, in, in_bytes, hipMemcpyHostToDevice, s) : hipSuccess;
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(H2D input)");
    std::vector<uint64_t> used(n, 0), cap(n), meta(7ull * n);  // meta: in_off, in_len, out_off, out_cap | len, cons, st
    std::vector<uint32_t> idx(n);
    std::vector<uint8_t> live(n);
    for (uint32_t c = 0; c < n; ++c) {
        live[c] = in_len[c] > 0;
        cap[c] = slot_guess[c] < 8 ? 8 : slot_guess[c];
        status[c] = CAPNP_PACKED_END_OF_STREAM;
    }
    uint64_t fcur = 0;  // bytes of `frames` used by earlier rounds
    uint32_t nf = 0;
    for (uint32_t r = 0;; ++r) {
        const uint32_t b = r & 1;  // this round's frame slots: d_out[b]
        // one round: the next message of every connection that may still hold one
        uint32_t k = 0;
        for (uint32_t c = 0; c < n; ++c)
            if (live[c] && used[c] < in_len[c]) idx[k++] = c;
        if (k == 0) break;
        uint64_t* const h_in_off = meta.data();
        uint64_t* const h_in_len = h_in_off + k;
        uint64_t* const h_out_off = h_in_off + 2 * k;
        uint64_t* const h_out_cap = h_in_off + 3 * k;
        uint64_t slots = 0;
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t c = idx[j];
            h_in_off[j] = in_off[c] + used[c];
            h_in_len[j] = in_len[c] - used[c];
            h_out_cap[j] = (cap[c] + 7) & ~7ull;
            h_out_off[j] = slots;
            slots += h_out_cap[j];
        }
        // round r - 2's frames left d_out[b] before it is reused (or reallocated)
        e = hipEventSynchronize(g_fr.ev_copied[b]);
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize(frames copy)");
        if ((st = g_fr.reserve(&g_fr.d_out[b], &g_fr.out_cap[b], slots + 16))) return st;
        uint64_t* const dm = reinterpret_cast<uint64_t*>(g_fr.d_meta);
        e = hipMemcpyAsync(dm, h_in_off, 4ull * k * sizeof(uint64_t), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(H2D round)");
        int32_t* const d_st = reinterpret_cast<int32_t*>(dm + 6ull * k);
        e = cpk::launch_read_message(g_fr.d_in, dm, dm + k, k, g_fr.d_out[b], dm + 2ull * k, dm + 3ull * k,
                                     dm + 4ull * k, dm + 5ull * k, d_st, s);
        if (e == hipSuccess) e = hipEventRecord(g_fr.ev_done[b], s);
        if (e != hipSuccess) return hip_fail(e, "read-message launch");
        uint64_t* const h_len = h_in_off + 4 * k;
        uint64_t* const h_cons = h_in_off + 5 * k;
        int32_t* const h_st = reinterpret_cast<int32_t*>(h_in_off + 6 * k);
        e = hipMemcpyAsync(h_len, dm + 4ull * k, 2ull * k * sizeof(uint64_t) + k * sizeof(int32_t),
                           hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(D2H round)");
        // the round's frames go to `frames` as one copy of its slots up to the last good one
        uint64_t span = 0;
        uint32_t good = 0;
        for (uint32_t j = 0; j < k; ++j)
            if (h_st[j] == CAPNP_PACKED_OK) {
                span = h_out_off[j] + h_len[j];
                ++good;
            }
        if (good) {
            if (fcur > frames_cap || span > frames_cap - fcur || good > max_frames - nf)
                return fail(CAPNP_PACKED_OUT_OF_SPACE, "frames buffer or frame table too small");
            // on the copy stream, while the next round decodes into the other buffer
            e = hipStreamWaitEvent(g_fr.copy, g_fr.ev_done[b], 0);
            if (e == hipSuccess) e = hipMemcpyAsync(frames + fcur, g_fr.d_out[b], span, hipMemcpyDeviceToHost, g_fr.copy);
            if (e == hipSuccess) e = hipEventRecord(g_fr.ev_copied[b], g_fr.copy);
            if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(D2H frames)");
        }
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t c = idx[j];
            const int32_t rs = h_st[j];
            if (rs == CAPNP_PACKED_OK) {
                frame_off[nf] = fcur + h_out_off[j];
                frame_len[nf] = h_len[j];
                frame_conn[nf] = c;
                ++nf;
                used[c] += h_cons[j];
                cap[c] = h_len[j] < 8 ? 8 : h_len[j];
            } else if (rs == CAPNP_PACKED_OUT_OF_SPACE) {
                // the reader reported the framed length: next round, a slot that holds it
                cap[c] = std::max(2 * cap[c], (uint64_t)h_len[j]);
            } else {
                live[c] = 0;  // END_OF_STREAM: the rest waits for the next read; else the error
                status[c] = rs;
            }
        }
        fcur += (span + 7) & ~7ull;
    }
    for (uint32_t c = 0; c < n; ++c) {
        consumed[c] = used[c];
        slot_guess[c] = cap[c];
    }
    *n_frames = nf;
    return CAPNP_PACKED_OK;
}

}  // extern "C"


// ---------------------------------------------------------------------------
// Resumable framing of packed socket streams: Connection.handleRead
// (src/rpc/level2/connection.zig:153-203) with Framer state kept across reads
// (src/rpc/level0/framing.zig:42-90 keeps expected_total; reader.zig:84-156 is one pass).
// Each connection's unconsumed packed bytes live in a region of one device arena, so a read
// uploads only its new bytes. Per connection the session keeps the current message's framed
// length (need, from read_header_kernel once its header is decoded) and where its walk
// stopped (X: packed bytes from the message start, W: words decoded), so the next read's
// walk (frame_walk_kernel) starts there: a message split over k reads is uploaded once and
// walked once. A complete message is decoded straight from the arena into its frame slot
// (the batch decoder) and copied to the caller's frames buffer.
//
// Regions: a connection's region is [off, off + cap) of the arena, its bytes [m0, len) of
// it. A read that does not fit moves the connection's bytes to a fresh region of twice their
// size at the arena top (the bytes of a partial message move once per doubling); when the
// top reaches the end, every connection's bytes move to a new arena of twice the live size.
// ---------------------------------------------------------------------------
struct capnp_packed_framer {
    std::mutex mu;
    uint32_t n = 0;
    hipStream_t s = nullptr;
    uint8_t* arena = nullptr;
    uint64_t acap = 0, top = 0;
    std::vector<uint64_t> off, cap, m0, len, need, X, W;  // per connection (host authoritative)
    // device scratch: per-connection arrays (base, avail, need, X, W, consumed, status),
    // lists and unit metadata of a round, copy jobs, the input staging and the frame slots
    uint8_t* d_state = nullptr;
    uint64_t state_cap = 0;
    uint8_t* d_stage = nullptr;
    uint64_t stage_cap = 0;
    uint8_t* d_frames = nullptr;
    uint64_t frames_dcap = 0;
    uint8_t* d_spec = nullptr;  // the walk's window tables (cpk::launch_frame_walk)
    uint64_t spec_cap = 0;
    uint8_t* d_round = nullptr;  // a walk pass's list, counts and message table
    uint64_t round_cap = 0;
    uint8_t* d_units = nullptr;  // a decode pass's unit metadata (6 u64 per message)
    uint64_t units_cap = 0;
    uint8_t* h_stage = nullptr;  // page-locked gather of capnp_packed_framer_readv's reads
    uint64_t h_stage_cap = 0;
    // page-locked host sides of a read's metadata copies: per-connection state, a walk pass's
    // counts and message table, a decode pass's unit metadata (no pageable staging per copy)
    struct Pinned {
        uint8_t* p = nullptr;
        uint64_t cap = 0;
        int reserve(uint64_t bytes) {
            if (p && bytes <= cap) return CAPNP_PACKED_OK;
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            const uint64_t want = std::max<uint64_t>(bytes + bytes / 2, 4096);
            const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), want, hipHostMallocDefault);
            if (e != hipSuccess) {
                p = nullptr;
                return hip_fail(e, "hipHostMalloc(framer metadata)");
            }
            cap = want;
            return CAPNP_PACKED_OK;
        }
        ~Pinned() {
            if (p) (void)hipHostFree(p);
        }
    } pin_state, pin_tab, pin_units, pin_jobs;
    uint64_t uploaded = 0, moved = 0;  // bytes copied H2D (new reads) and moved between regions
    int dev = -1;                      // the device the session was created on
    static constexpr uint32_t kWalkMessages = 64;  // messages a walk pass finds per connection

    ~capnp_packed_framer() {
        // the session's device is current for the teardown, whatever device the caller has
        // current now (the library's stream contexts are keyed by device and stream)
        int cur = -1;
        const bool switched = dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev &&
                              hipSetDevice(dev) == hipSuccess;
        if (s) {
            (void)hipStreamSynchronize(s);
            // the decode passes ran on s: drop the library's context of it (side stream, events,
            // class queue), or every session ever created would keep one
            (void)cpk::release_stream(s, dev);
        }
        if (arena) (void)hipFree(arena);
        if (d_state) (void)hipFree(d_state);
        if (d_stage) (void)hipFree(d_stage);
        if (d_frames) (void)hipFree(d_frames);
        if (d_spec) (void)hipFree(d_spec);
        if (d_round) (void)hipFree(d_round);
        if (d_units) (void)hipFree(d_units);
        if (h_stage) (void)hipHostFree(h_stage);
        if (s) (void)hipStreamDestroy(s);
        if (switched) (void)hipSetDevice(cur);
    }
    static int grow(uint8_t** p, uint64_t* c, uint64_t need) {
        if (*p && need <= *c) return CAPNP_PACKED_OK;
        const uint64_t want = need < 65536 ? 65536 : need + need / 2;
        if (*p) (void)hipFree(*p);
        *p = nullptr;
        *c = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(p), want);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(framer session)");
        *c = want;
        return CAPNP_PACKED_OK;
    }
    // The copy jobs of a read (host vector hjobs, kept until the stream has consumed it, so a
    // read's upload and region copies need no synchronisation of their own: the walk pass's
    // synchronisation covers them).
    std::vector<uint64_t> hjobs;
    bool jobs_inflight = false;
    int settle() {  // the previous read's job upload is done with hjobs
        if (!jobs_inflight) return CAPNP_PACKED_OK;
        jobs_inflight = false;
        const hipError_t e = hipStreamSynchronize(s);
        return e == hipSuccess ? CAPNP_PACKED_OK : hip_fail(e, "framer copy jobs");
    }
    // The first `first` jobs run as a launch of their own, before the others (stream order).
    int run_jobs(std::vector<uint64_t>& jobs, bool wait = true, uint32_t first = 0) {
        if (jobs.empty()) return CAPNP_PACKED_OK;
        const uint32_t nj = (uint32_t)(jobs.size() / 3);
        // the jobs go after the per-connection arrays in the state scratch
        const uint64_t at = (uint64_t)n * 56 + 256;
        int st = grow(&d_state, &state_cap, at + jobs.size() * 8 + 64 * (uint64_t)n + 4096);
        if (st) return st;
        uint64_t* const dj = reinterpret_cast<uint64_t*>(d_state + at);
        if ((st = pin_jobs.reserve(jobs.size() * 8))) return st;  // page-locked: no staged copy
        std::memcpy(pin_jobs.p, jobs.data(), jobs.size() * 8);
        hipError_t e = hipMemcpyAsync(dj, pin_jobs.p, jobs.size() * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && first) e = cpk::launch_copy_jobs(dj, first, s);
        if (e == hipSuccess) e = cpk::launch_copy_jobs(dj + 3ull * first, nj - first, s);
        if (e == hipSuccess && wait) e = hipStreamSynchronize(s);  // `jobs` is reused by the caller
        if (e != hipSuccess) return hip_fail(e, "framer copy jobs");
        if (wait) jobs.clear();
        else jobs_inflight = true;  // hjobs only: cleared by the next read after settle()
        return CAPNP_PACKED_OK;
    }
    static uint64_t region_for(uint64_t bytes) { return std::max<uint64_t>(65536, (2 * bytes + 255) & ~255ull); }
    // A read's region layout, built on copies and committed (commit) only once every copy job
    // of the read is enqueued: a failed allocation or launch leaves the session as it was.
    struct Layout {
        std::vector<uint64_t> off, cap, m0, len;
        uint64_t top = 0, moved = 0;
        uint8_t* arena = nullptr;  // a new arena (rearena), freed unless committed
        uint64_t acap = 0;
        ~Layout() {
            if (arena) (void)hipFree(arena);
        }
    };
    void commit(Layout& L) {
        off.swap(L.off);
        cap.swap(L.cap);
        m0.swap(L.m0);
        len.swap(L.len);
        top = L.top;
        moved = L.moved;
        if (L.arena) {
            if (arena) (void)hipFree(arena);
            arena = L.arena;
            acap = L.acap;
            L.arena = nullptr;
        }
    }
    // Every connection's live bytes into a new arena (L.arena) with a region sized for want[c]
    // bytes each; the moves run (and complete) now, from the current arena, which stays valid.
    int rearena(const std::vector<uint64_t>& want, Layout& L) {
        uint64_t total = 0;
        for (uint32_t c = 0; c < n; ++c) total += want[c] ? region_for(want[c]) : 0;
        const uint64_t ncap = std::max<uint64_t>(2 * total, 1u << 20);
        uint8_t* na = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&na), ncap + 64);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(framer arena)");
        L.arena = na;
        L.acap = ncap;
        std::vector<uint64_t> jobs;
        uint64_t t = 0;
        for (uint32_t c = 0; c < n; ++c) {
            const uint64_t live = L.len[c] - L.m0[c];
            if (!want[c]) {
                L.off[c] = L.cap[c] = L.m0[c] = L.len[c] = 0;
                continue;
            }
            const uint64_t rc = region_for(want[c]);
            if (live) {
                jobs.insert(jobs.end(), {reinterpret_cast<uint64_t>(na + t), reinterpret_cast<uint64_t>(arena + L.off[c] + L.m0[c]), live});
                L.moved += live;
            }
            L.off[c] = t;
            L.cap[c] = rc;
            L.m0[c] = 0;
            L.len[c] = live;
            t += rc;
        }
        L.top = t;
        return run_jobs(jobs);
    }
};

namespace {

int framer_check(capnp_packed_framer* f, uint32_t conn) {
    if (!f) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "framer is null");
    if (conn >= f->n) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "connection index out of range");
    return CAPNP_PACKED_OK;
}

}  // namespace

extern "C" {

int capnp_packed_framer_create(uint32_t n_conns, capnp_packed_framer** out) {
    if (!out) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "out is null");
    *out = nullptr;
    if (n_conns == 0) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "a framer needs at least one connection");
    int st = ensure_device();
    if (st) return st;
    capnp_packed_framer* f = new (std::nothrow) capnp_packed_framer();
    if (!f) return fail(CAPNP_PACKED_OUT_OF_SPACE, "framer allocation");
    f->n = n_conns;
    if (hipGetDevice(&f->dev) != hipSuccess) f->dev = -1;
    for (auto* v : {&f->off, &f->cap, &f->m0, &f->len, &f->need, &f->X, &f->W}) v->assign(n_conns, 0);
    hipError_t e = hipStreamCreateWithFlags(&f->s, hipStreamNonBlocking);
    if (e != hipSuccess) {
        f->s = nullptr;
        delete f;
        return hip_fail(e, "hipStreamCreate(framer session)");
    }
    *out = f;
    return CAPNP_PACKED_OK;
}

int capnp_packed_framer_destroy(capnp_packed_framer* f) {
    if (!f) return CAPNP_PACKED_OK;
    delete f;  // synchronises its stream first
    return CAPNP_PACKED_OK;
}

int capnp_packed_framer_reset(capnp_packed_framer* f, uint32_t conn) {
    int st = framer_check(f, conn);
    if (st) return st;
    std::lock_guard<std::mutex> lock(f->mu);
    f->m0[conn] = f->len[conn] = 0;
    f->need[conn] = f->X[conn] = f->W[conn] = 0;
    return CAPNP_PACKED_OK;
}

int capnp_packed_framer_buffered(capnp_packed_framer* f, uint32_t conn, uint64_t* bytes) {
    int st = framer_check(f, conn);
    if (st) return st;
    if (!bytes) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "bytes is null");
    std::lock_guard<std::mutex> lock(f->mu);
    *bytes = f->len[conn] - f->m0[conn];
    return CAPNP_PACKED_OK;
}

int capnp_packed_framer_expected(capnp_packed_framer* f, uint32_t conn, uint64_t* framed_bytes) {
    int st = framer_check(f, conn);
    if (st) return st;
    if (!framed_bytes) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "framed_bytes is null");
    std::lock_guard<std::mutex> lock(f->mu);
    *framed_bytes = f->need[conn];
    return CAPNP_PACKED_OK;
}

int capnp_packed_framer_stats(capnp_packed_framer* f, uint64_t* uploaded, uint64_t* moved) {
    if (!f || !uploaded || !moved) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null pointer");
    std::lock_guard<std::mutex> lock(f->mu);
    *uploaded = f->uploaded;
    *moved = f->moved;
    return CAPNP_PACKED_OK;
}

}  // extern "C"

namespace {


// The gather of capnp_packed_framer_readv: bytes [r0, r1) of the connections' reads, laid end
// to end at their prefix offsets, into the session's page-locked staging, by byte range over up
// to 8 threads from 4 MiB up.
void gather_reads(uint8_t* dst, const uint8_t* const* ptr, const uint64_t* len, const uint64_t* off, uint32_t n,
                  uint64_t r0, uint64_t r1) {
    auto copy_range = [=](uint64_t b0, uint64_t b1) {
        // the first connection whose bytes end past b0
        uint32_t c = (uint32_t)(std::upper_bound(off, off + n, b0) - off);
        c = c ? c - 1 : 0;
        for (; c < n && off[c] < b1; ++c) {
            if (!len[c]) continue;
            const uint64_t lo = std::max(off[c], b0), hi = std::min(off[c] + len[c], b1);
            if (lo < hi) std::memcpy(dst + lo, ptr[c] + (lo - off[c]), hi - lo);
        }
    };
    const uint64_t total = r1 - r0;
    const unsigned hw = std::thread::hardware_concurrency();
    const unsigned T = total < (4ull << 20) ? 1u : std::max(1u, std::min(8u, hw ? hw : 1u));
    std::vector<std::thread> th;
    try {
        for (unsigned t = 1; t < T; ++t) th.emplace_back(copy_range, r0 + total * t / T, r0 + total * (t + 1) / T);
    } catch (...) {  // no threads: the rest on this one
        copy_range(r0 + total * (th.size() + 1) / T, r1);
    }
    copy_range(r0, r0 + total / T);
    for (auto& x : th) x.join();
}

int framer_args(capnp_packed_framer* f, uint8_t* frames, uint64_t frames_cap, uint64_t* frame_off,
                uint64_t* frame_len, uint32_t* frame_conn, uint32_t max_frames, int32_t* status, uint32_t* n_frames) {
    if (!n_frames) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "n_frames is null");
    *n_frames = 0;
    if (!f) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "framer is null");
    if (!status || (max_frames && (!frame_off || !frame_len || !frame_conn)) || (frames_cap && !frames))
        return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null pointer");
    return CAPNP_PACKED_OK;
}

// capnp_packed_framer_read with f->mu held and its arguments checked
// (staged: the caller already put the input's bytes into d_stage on the session's stream)
int framer_read_locked(capnp_packed_framer* f, const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                       const uint64_t* in_len, uint8_t* frames, uint64_t frames_cap, uint64_t* frame_off,
                       uint64_t* frame_len, uint32_t* frame_conn, uint32_t max_frames, int32_t* status,
                       uint32_t* n_frames, bool staged = false) {
    const uint32_t n = f->n;
    const hipStream_t s = f->s;
    hipError_t e = hipSuccess;
    int st = CAPNP_PACKED_OK;
    for (uint32_t c = 0; c < n; ++c) status[c] = CAPNP_PACKED_END_OF_STREAM;

    // ---- 1. the new bytes: one H2D into the staging buffer, appended to the regions ---------
    if ((st = f->settle())) return st;  // a previous read's copies are done with d_stage / hjobs
    if (in_bytes && in_len) {
        if (!staged) {
            if ((st = capnp_packed_framer::grow(&f->d_stage, &f->stage_cap, in_bytes + 32))) return st;
            e = hipMemcpyAsync(f->d_stage, in, in_bytes, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(framer H2D)");
        }
        // regions: a connection whose bytes would pass its region's end slides its held bytes to
        // the region's start when they and the new bytes fit there and the slide's source and
        // target do not overlap (held <= m0; a drained connection just restarts there), else it
        // gets a new region. The slides run as a launch of their own before the appends, which may
        // overwrite their source.
        auto slides = [&](uint32_t c) {
            const uint64_t held = f->len[c] - f->m0[c];
            return in_len[c] && f->len[c] + in_len[c] > f->cap[c] && held + in_len[c] <= f->cap[c] && held <= f->m0[c];
        };  // (on the session's layout, before this read)
        std::vector<uint64_t> want(n, 0);
        uint64_t grow_bytes = 0;
        bool any_grow = false;
        for (uint32_t c = 0; c < n; ++c) {
            const uint64_t live = f->len[c] - f->m0[c] + in_len[c];
            want[c] = live;
            if (in_len[c] && f->len[c] + in_len[c] > f->cap[c] && !slides(c)) {
                any_grow = true;
                grow_bytes += capnp_packed_framer::region_for(live);
            }
        }
        capnp_packed_framer::Layout L;  // the session's layout after this read, committed below
        L.off = f->off;
        L.cap = f->cap;
        L.m0 = f->m0;
        L.len = f->len;
        L.top = f->top;
        L.moved = f->moved;
        std::vector<uint64_t>& jobs = f->hjobs;
        jobs.clear();
        uint32_t n_slides = 0;
        if (any_grow && f->top + grow_bytes > f->acap) {
            if ((st = f->rearena(want, L))) return st;  // every region sized for its bytes after this read
        } else {
            for (uint32_t c = 0; c < n; ++c) {
                if (!slides(c)) continue;
                const uint64_t held = L.len[c] - L.m0[c];
                if (held) {
                    jobs.insert(jobs.end(), {reinterpret_cast<uint64_t>(f->arena + L.off[c]),
                                             reinterpret_cast<uint64_t>(f->arena + L.off[c] + L.m0[c]), held});
                    L.moved += held;
                    ++n_slides;
                }
                L.m0[c] = 0;
                L.len[c] = held;
            }
            for (uint32_t c = 0; any_grow && c < n; ++c) {  // the slid ones fit now
                if (!in_len[c] || L.len[c] + in_len[c] <= L.cap[c]) continue;
                const uint64_t live = L.len[c] - L.m0[c];
                const uint64_t rc = capnp_packed_framer::region_for(want[c]);
                if (live) {
                    jobs.insert(jobs.end(), {reinterpret_cast<uint64_t>(f->arena + L.top),
                                             reinterpret_cast<uint64_t>(f->arena + L.off[c] + L.m0[c]), live});
                    L.moved += live;
                }
                L.off[c] = L.top;
                L.cap[c] = rc;
                L.m0[c] = 0;
                L.len[c] = live;
                L.top += rc;
            }
        }
        for (uint32_t c = 0; c < n; ++c) {
            if (!in_len[c]) continue;
            jobs.insert(jobs.end(), {reinterpret_cast<uint64_t>((L.arena ? L.arena : f->arena) + L.off[c] + L.len[c]),
                                     reinterpret_cast<uint64_t>(f->d_stage + in_off[c]), in_len[c]});
            L.len[c] += in_len[c];
        }
        if ((st = f->run_jobs(jobs, false, n_slides))) return st;  // ordered before the passes below
        f->commit(L);  // every copy of this read is enqueued: the regions describe the arena now
        f->uploaded += in_bytes;
    }

    // ---- 2. passes: a walk over every connection's held messages, then one decode of them ----
    // state scratch: base, avail, need, X, W (u64 x n), status (i32 x n), then the copy jobs
    // (run_jobs) past them; the pass's list / counts / message table and the decode metadata
    // live in blocks of their own
    if ((st = capnp_packed_framer::grow(&f->d_state, &f->state_cap, (uint64_t)n * 56 + 256 + 64ull * n + 4096))) return st;
    uint64_t* const d_base = reinterpret_cast<uint64_t*>(f->d_state);
    uint64_t* const d_avail = d_base + n;
    uint64_t* const d_need = d_base + 2ull * n;
    uint64_t* const d_X = d_base + 3ull * n;
    uint64_t* const d_W = d_base + 4ull * n;
    int32_t* const d_st = reinterpret_cast<int32_t*>(d_base + 6ull * n);
    constexpr uint32_t M = capnp_packed_framer::kWalkMessages;
    if ((st = f->pin_state.reserve(60ull * n))) return st;  // 7 u64 then the pass's list (u32) per connection
    uint64_t* const h = reinterpret_cast<uint64_t*>(f->pin_state.p);  // base, avail, need, X, W, (free), status (i32)
    std::vector<uint32_t> spec_h;    // window tables' first / count per listed connection
    std::vector<uint64_t> spec_h64;  // their bytes: arena offset, length
    uint64_t spec_T = 0;
    const int32_t* const hst = reinterpret_cast<const int32_t*>(h + 6ull * n);
    std::vector<uint32_t> list;
    std::vector<uint8_t> dead(n, 0), more(n, 0);  // dead: an error this call (the connection was reset)
    std::vector<uint64_t> adv(n), um;             // adv: packed bytes of the pass's accepted messages
    std::vector<uint32_t> uconn;                  // the pass's accepted messages: connection
    std::vector<int32_t> perr(n);                 // an error to report once the pass's frames are out
    for (uint32_t c = 0; c < n; ++c) more[c] = f->len[c] > f->m0[c];
    uint64_t fcur = 0;
    uint32_t nf = 0;
    auto fail_conn = [&](uint32_t c, int32_t code) {
        status[c] = code;
        dead[c] = 1;
        f->m0[c] = f->len[c] = 0;  // Connection.handleRead resets the framer (connection.zig:175-184)
        f->need[c] = f->X[c] = f->W[c] = 0;
    };
    bool full = false;
    while (!full) {
        list.clear();
        for (uint32_t c = 0; c < n; ++c)
            if (!dead[c] && more[c]) list.push_back(c);
        uint32_t k = (uint32_t)list.size();
        if (k == 0) break;
        for (uint32_t c = 0; c < n; ++c) {
            h[c] = f->off[c] + f->m0[c];
            h[n + c] = f->len[c] - f->m0[c];
            h[2ull * n + c] = f->need[c];
            h[3ull * n + c] = f->X[c];
            h[4ull * n + c] = f->W[c];
        }
        const uint64_t tab_words = 2ull * k * M;
        if ((st = capnp_packed_framer::grow(&f->d_round, &f->round_cap, 4ull * (2ull * k + tab_words) + 256))) return st;
        uint32_t* const r_list = reinterpret_cast<uint32_t*>(f->d_round);
        uint32_t* const r_cnt = r_list + k;
        uint32_t* const r_tab = r_cnt + k;
        // window tables for the connections whose walk will cross whole windows inside one
        // message (crossed by lookups): the current message's framed bytes still to walk span
        // more than two windows, or, with its header not decoded yet, the held bytes span 64
        // windows. Many small messages end in nearly every window, where a table only costs.
        const uint64_t wb = cpk::framer_window_bytes(), wcap = cpk::framer_window_cap(k);
        spec_h.assign(2ull * k, 0);  // first, count per listed connection (u32); off, len (u64) below
        spec_h64.assign(2ull * k, 0);
        uint64_t T = 0;
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t c = list[j];
            const uint64_t span = f->len[c] - f->m0[c] - f->X[c];
            const uint64_t left = f->need[c] > 8 * f->W[c] ? f->need[c] - 8 * f->W[c] : 0;
            const bool lookups = f->need[c] ? left > 2 * wb : span > 64 * wb;
            uint64_t cnt = lookups && span > wb ? (span + wb - 1) / wb : 0;
            if (T + cnt > wcap) cnt = 0;
            spec_h[j] = cnt ? (uint32_t)T : 0xFFFFFFFFu;
            spec_h[k + j] = (uint32_t)cnt;
            spec_h64[j] = f->off[c] + f->m0[c] + f->X[c];
            spec_h64[k + j] = span;
            T += cnt;
        }
        uint32_t* d_sq = nullptr;
        const uint32_t *d_sfirst = nullptr, *d_scount = nullptr;
        const uint64_t *d_soff = nullptr, *d_slen = nullptr;
        if (T) {
            const uint64_t qb = (cpk::framer_spec_bytes(k, T) + 15) & ~15ull;
            const uint64_t ab = (8ull * k + 15) & ~15ull;
            if ((st = capnp_packed_framer::grow(&f->d_spec, &f->spec_cap, qb + ab + 16ull * k + 64))) return st;
            d_sq = reinterpret_cast<uint32_t*>(f->d_spec);
            uint32_t* const a32 = reinterpret_cast<uint32_t*>(f->d_spec + qb);
            uint64_t* const a64 = reinterpret_cast<uint64_t*>(f->d_spec + qb + ab);
            d_sfirst = a32;
            d_scount = a32 + k;
            d_soff = a64;
            d_slen = a64 + k;
            spec_T = T;
            e = hipMemcpyAsync(d_sq + 8, &spec_T, 8, hipMemcpyHostToDevice, s);  // q_tiles: the windows
            if (e == hipSuccess) e = hipMemcpyAsync(a32, spec_h.data(), 8ull * k, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = hipMemcpyAsync(a64, spec_h64.data(), 16ull * k, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) return hip_fail(e, "framer window tables");
        }
        if ((st = f->pin_tab.reserve(4ull * (k + tab_words)))) return st;
        const uint32_t* const hcnt = reinterpret_cast<const uint32_t*>(f->pin_tab.p);  // counts, then the table
        e = hipMemcpyAsync(d_base, h, 5ull * n * 8, hipMemcpyHostToDevice, s);
        uint32_t* const plist = reinterpret_cast<uint32_t*>(f->pin_state.p + 56ull * n);
        std::memcpy(plist, list.data(), 4ull * k);
        if (e == hipSuccess) e = hipMemcpyAsync(r_list, plist, 4ull * k, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = cpk::launch_frame_walk(f->arena, r_list, k, d_base, d_avail, d_need, d_X, d_W, d_st, M, r_cnt, r_tab,
                                       d_sq, T, d_sfirst, d_scount, d_soff, d_slen, s);
        // need, X, W, (a free slot), status: one copy; the counts and the table: another
        if (e == hipSuccess) e = hipMemcpyAsync(h + 2ull * n, d_need, 3ull * n * 8 + n * 8 + 4ull * n, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(f->pin_tab.p, r_cnt, 4ull * (k + tab_words), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "framer walk pass");
        f->jobs_inflight = false;
        // whole messages, in order per connection, while the frames buffer and table hold them:
        // decoded from the arena into frame slots, then to the caller's buffer
        um.clear();  // per message: in_off, in_len, out_off, out_cap
        uconn.clear();
        uint64_t slots = 0;
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t c = list[j];
            const uint32_t* const tj = hcnt + k + 2ull * j * M;
            uint64_t at = 0;
            uint32_t m = 0;
            for (; m < hcnt[j]; ++m) {
                const uint64_t L = tj[2 * m + 1];
                if (nf + uconn.size() + 1 > max_frames || fcur + slots + L > frames_cap) {
                    full = true;  // stays whole in its region: the next call pops it
                    break;
                }
                um.insert(um.end(), {f->off[c] + f->m0[c] + at, tj[2 * m], slots, L});
                uconn.push_back(c);
                slots += (L + 7) & ~7ull;
                at += tj[2 * m];
            }
            adv[c] = at;
            perr[c] = CAPNP_PACKED_OK;
            more[c] = 0;
            if (m < hcnt[j]) {  // the frames ran out: message m stays found whole (X at its end)
                h[2ull * n + c] = tj[2 * m + 1];
                h[3ull * n + c] = tj[2 * m];
                h[4ull * n + c] = tj[2 * m + 1] / 8;
            } else if (hst[c] == CAPNP_PACKED_OK) {
                more[c] = 1;  // M messages: the next pass walks on from the last one's end
            } else if (hst[c] != CAPNP_PACKED_END_OF_STREAM) {
                perr[c] = hst[c];
            }
        }
        const uint32_t U = (uint32_t)uconn.size();
        if (U) {
            if ((st = capnp_packed_framer::grow(&f->d_frames, &f->frames_dcap, slots + 16))) return st;
            if ((st = capnp_packed_framer::grow(&f->d_units, &f->units_cap, 48ull * U + 64))) return st;
            uint64_t* const u = reinterpret_cast<uint64_t*>(f->d_units);
            if ((st = f->pin_units.reserve(48ull * U))) return st;
            uint64_t* const hm = reinterpret_cast<uint64_t*>(f->pin_units.p);
            for (uint32_t q = 0; q < U; ++q)
                for (uint32_t a = 0; a < 4; ++a) hm[a * (uint64_t)U + q] = um[4ull * q + a];
            e = hipMemcpyAsync(u, hm, 4ull * U * 8, hipMemcpyHostToDevice, s);
            int32_t* const u_st = reinterpret_cast<int32_t*>(u + 5ull * U);
            if (e == hipSuccess)
                e = cpk::launch_decode(f->arena, u, u + U, U, f->d_frames, u + 2ull * U, u + 3ull * U, u + 4ull * U,
                                       u_st, true, nullptr, 0, s);
            if (e == hipSuccess) e = hipMemcpyAsync(frames + fcur, f->d_frames, slots, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipMemcpyAsync(hm + 4ull * U, u + 4ull * U, 2ull * U * 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) return hip_fail(e, "framer decode pass");
            const int32_t* const us = reinterpret_cast<const int32_t*>(hm + 5ull * U);
            for (uint32_t q = 0; q < U; ++q) {
                if (us[q] != CAPNP_PACKED_OK || hm[4ull * U + q] != hm[3ull * U + q])  // the walk verified the bytes
                    return fail(CAPNP_PACKED_DEVICE_ERROR, "framer: a walked message did not decode to its framed length");
                frame_off[nf] = fcur + hm[2ull * U + q];
                frame_len[nf] = hm[3ull * U + q];
                frame_conn[nf] = uconn[q];
                ++nf;
            }
            fcur += slots;
        }
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t c = list[j];
            f->m0[c] += adv[c];
            f->need[c] = h[2ull * n + c];
            f->X[c] = h[3ull * n + c];
            f->W[c] = h[4ull * n + c];
            if (perr[c] != CAPNP_PACKED_OK) fail_conn(c, perr[c]);  // after the frames before it
        }
    }
    *n_frames = nf;
    if ((st = f->settle())) return st;  // no pass ran after the upload: the caller's bytes are consumed
    return full ? fail(CAPNP_PACKED_OUT_OF_SPACE, "frames buffer or frame table full: call again to pop the rest")
                : CAPNP_PACKED_OK;
}

}  // namespace

extern "C" {

int capnp_packed_framer_read(capnp_packed_framer* f, const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                             const uint64_t* in_len, uint8_t* frames, uint64_t frames_cap, uint64_t* frame_off,
                             uint64_t* frame_len, uint32_t* frame_conn, uint32_t max_frames, int32_t* status,
                             uint32_t* n_frames) {
    int st = framer_args(f, frames, frames_cap, frame_off, frame_len, frame_conn, max_frames, status, n_frames);
    if (st) return st;
    const uint32_t n = f->n;
    if (in_bytes && (!in || !in_off || !in_len)) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null pointer");
    if (in_len)
        for (uint32_t c = 0; c < n; ++c)
            if (in_len[c] && (!in_off || in_off[c] > in_bytes || in_len[c] > in_bytes - in_off[c]))
                return fail(CAPNP_PACKED_INVALID_ARGUMENT, "connection bytes outside the input buffer");
    std::lock_guard<std::mutex> lock(f->mu);
    return framer_read_locked(f, in, in_bytes, in_off, in_len, frames, frames_cap, frame_off, frame_len, frame_conn,
                              max_frames, status, n_frames);
}

int capnp_packed_framer_readv(capnp_packed_framer* f, const uint8_t* const* in_ptr, const uint64_t* in_len,
                              uint8_t* frames, uint64_t frames_cap, uint64_t* frame_off, uint64_t* frame_len,
                              uint32_t* frame_conn, uint32_t max_frames, int32_t* status, uint32_t* n_frames) {
    int st = framer_args(f, frames, frames_cap, frame_off, frame_len, frame_conn, max_frames, status, n_frames);
    if (st) return st;
    const uint32_t n = f->n;
    if (!in_ptr || !in_len) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "null pointer");
    std::vector<uint64_t> off(n);
    uint64_t total = 0;
    for (uint32_t c = 0; c < n; ++c) {
        if (in_len[c] && !in_ptr[c]) return fail(CAPNP_PACKED_INVALID_ARGUMENT, "a connection's bytes are null");
        off[c] = total;
        total += in_len[c];
    }
    std::lock_guard<std::mutex> lock(f->mu);
    if (total) {
        // the previous call's upload from the staging has finished (each call ends synchronised)
        if (!f->h_stage || f->h_stage_cap < total) {
            if (f->h_stage) (void)hipHostFree(f->h_stage);
            f->h_stage = nullptr;
            f->h_stage_cap = 0;
            const uint64_t want = std::max<uint64_t>(total + total / 4, 1u << 20);
            hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&f->h_stage), want, hipHostMallocDefault);
            if (e != hipSuccess) {
                f->h_stage = nullptr;
                return hip_fail(e, "hipHostMalloc(framer staging)");
            }
            f->h_stage_cap = want;
        }
        // gather and upload in 32-MiB pieces: piece i's H2D runs while piece i + 1 is gathered
        if ((st = f->settle())) return st;  // the previous read's copies are done with d_stage
        if ((st = capnp_packed_framer::grow(&f->d_stage, &f->stage_cap, total + 32))) return st;
        constexpr uint64_t kPiece = 32ull << 20;
        for (uint64_t r0 = 0; r0 < total; r0 += kPiece) {
            const uint64_t r1 = std::min(total, r0 + kPiece);
            gather_reads(f->h_stage, in_ptr, in_len, off.data(), n, r0, r1);
            const hipError_t e = hipMemcpyAsync(f->d_stage + r0, f->h_stage + r0, r1 - r0, hipMemcpyHostToDevice, f->s);
            if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(framer H2D)");
        }
    }
    return framer_read_locked(f, total ? f->h_stage : nullptr, total, total ? off.data() : nullptr,
                              total ? in_len : nullptr, frames, frames_cap, frame_off, frame_len, frame_conn,
                              max_frames, status, n_frames, true);
}

}  // extern "C"
