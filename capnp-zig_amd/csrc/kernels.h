// kernels.h — internal launcher interface between the C-ABI (capnp_packed_abi.cpp)
// and the gfx950 kernels (packed_kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace cpk {

// Batch encode / decode (write = false: sizes only). ws: optional caller workspace of
// at least queue_bytes(n) bytes for the long-unit queue (nullptr: the caller stream's
// own queue, kept by the library).
hipError_t launch_encode(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                         int32_t* status, bool write, void* ws, size_t ws_bytes, hipStream_t stream);

hipError_t launch_decode(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                         int32_t* status, bool write, void* ws, size_t ws_bytes, hipStream_t stream);

size_t queue_bytes(uint32_t n);

// capnp_packed_set_decoder: returns the previous setting
int set_decoder(int decoder);
bool decoder_built(int decoder);  // AUTO, TWO_PASS, WORDS (FUSED / STREAM removed in round 5)
int set_all_or_nothing(int on);
uint32_t set_launch_flags(uint32_t flags);
hipError_t release_stream(hipStream_t stream, int dev = -1);  // dev -1: the current device
void stream_queue_info(hipStream_t stream, size_t* bytes, uint32_t* kept);
uint32_t stream_context_count();  // caller streams with a library context (current device)

// Reader.readPackedMessage over a batch of reader streams (reader.zig:84-156).
// One unit (the single-buffer calls): the unit's status must be kStNeedFull (decode_one_status())
// for decode_one; encode_one takes units of at most 512 words.
int32_t decode_one_status();
hipError_t launch_decode_one(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                             hipStream_t stream);
hipError_t launch_encode_one(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len, int32_t* status,
                             bool write, hipStream_t stream);
hipError_t launch_read_message(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                               uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_len,
                               uint64_t* consumed, int32_t* status, hipStream_t stream);

// Resumable packed framing (capnp_packed_framer_*): batched device byte copies (3 u64 per job:
// dst, src, len), the header pass of Reader.readPackedMessage (framed length per unit), and the
// walk of each listed connection's message from its saved position.
hipError_t launch_copy_jobs(const uint64_t* jobs, uint32_t nj, hipStream_t stream);
hipError_t launch_read_header(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                              uint64_t* out_len, uint64_t* consumed, int32_t* status, hipStream_t stream);
// Framer walk (capnp_packed_framer_read): spec_q (framer_spec_bytes(nl, windows) bytes, u64 at
// u32 index 8 = windows) holds the window tables of the listed connections whose held bytes
// span more than one window (spec_first / spec_count per list entry, spec_off / spec_len their
// bytes from the walk's start); spec_q null or windows 0: every window walked exactly.
size_t framer_spec_bytes(uint32_t nl, uint64_t windows);
uint32_t framer_window_bytes();            // the windows' size (kWvWin)
uint64_t framer_window_cap(uint32_t nl);   // windows a spec table of nl connections may hold
// The walk goes on message after message, up to M per connection: cnt[i] messages found, their
// packed and framed lengths at tab[2 (i M + m)] / [+ 1] (u32); need / X / W / status then hold
// the current message's state (frame_walk_kernel).
hipError_t launch_frame_walk(const uint8_t* arena, const uint32_t* list, uint32_t nl, const uint64_t* base,
                             const uint64_t* avail, uint64_t* need, uint64_t* X, uint64_t* W, int32_t* status,
                             uint32_t M, uint32_t* cnt, uint32_t* tab, uint32_t* spec_q, uint64_t windows,
                             const uint32_t* spec_first, const uint32_t* spec_count, const uint64_t* spec_off,
                             const uint64_t* spec_len, hipStream_t stream);

// MessageBuilder.toPackedBytes from segment lists (message.zig:2123-2179).
hipError_t launch_encode_message(const uint64_t* seg_ptr, const uint64_t* seg_len, const uint32_t* seg_first,
                                 const uint32_t* seg_count, uint32_t n, uint8_t* out, const uint64_t* out_off,
                                 const uint64_t* out_cap, uint64_t* out_len, int32_t* status, bool write,
                                 hipStream_t stream);

// Message.init segment-table parse (message.zig:341-394).
hipError_t launch_message_init(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                               uint32_t max_segs, uint32_t* seg_count, uint64_t* seg_off, uint64_t* seg_len,
                               int32_t* status, hipStream_t stream);

// Message.validate (message.zig:699-969) of framed messages.
hipError_t launch_validate(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint32_t n,
                           uint64_t seg_limit, uint64_t trav_limit, uint32_t nest_limit, int32_t* status,
                           uint64_t* words, hipStream_t stream);

hipError_t launch_generate(uint8_t* out, uint64_t n_units, uint64_t unit_bytes, uint64_t unit_base,
                           uint64_t seed, uint32_t thr, hipStream_t stream);

size_t scan_scratch_bytes(uint32_t n);

hipError_t launch_scan(const uint64_t* len, uint32_t n, uint64_t base, uint64_t* off, uint64_t* scratch,
                       hipStream_t stream);

}  // namespace cpk
