/*
 * packed_oracle.h — CPU restatement of the reference Zig packed codec.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the
 * reported CPU baseline. The product path (capnp-zig_amd/) never links it.
 *
 * Pinning: the decoder is pinned by the reference's committed fixture pairs
 * (tests/capnp_testdata/testdata/{binary,packed,segmented,segmented-packed},
 * tests/interop/fixture_{single,far}[_packed].bin) and the known-answer tests
 * message.zig:2318-2349, reader.zig:304-386; the encoder is pinned by the
 * reference source (message.zig:200-271) and an independent Python
 * restatement (tests/pyref.py). No reference binary can be built here (Zig and
 * the libxev URL dependency are absent), so oracle/_ref does not exist: see
 * DESIGN.md §3.
 *
 * Status codes are the ones of include/capnp_packed.h.
 */
#ifndef PACKED_ORACLE_H
#define PACKED_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* message.zig:196-198 wordHasZeroByte */
int oracle_word_has_zero_byte(uint64_t v);

/* message.zig:200-271 packPacked. out may be NULL when cap == 0 (size query). */
int oracle_pack(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* message.zig:152-191 estimateUnpackedSize */
int oracle_estimate_unpacked_size(const uint8_t* in, size_t n, size_t* out_size);

/* message.zig:88-145 unpackPacked */
int oracle_unpack(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* message.zig:341-394 Message.init segment-table parse. Fills seg_off/seg_len
 * (capacity max_segs) and *seg_count. Returns 0 on success or a negative code:
 * -1 EndOfStream, -2 InvalidSegmentCount, -3 SegmentCountLimitExceeded,
 * -4 TruncatedMessage, -5 InvalidMessageSize. */
int oracle_message_init(const uint8_t* data, size_t n, uint32_t max_segs,
                        uint64_t* seg_off, uint64_t* seg_len, uint32_t* seg_count);

/* reader.zig:84-156 Reader.readPackedMessage over an in-memory stream.
 * *consumed = packed bytes read. Returns 0 or a negative code:
 * -1 EndOfStream, -2 InvalidSegmentCount, -3 SegmentCountLimitExceeded,
 * -6 MessageTooLarge, -7 InvalidPackedMessage, -8 OutOfSpace. */
int oracle_read_packed_message(const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                               size_t* out_len, size_t* consumed);
/* Connection.handleRead's loop over one connection's bytes (readPackedMessage until no whole
 * message is left); returns the frames read. */
size_t oracle_read_stream(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* used,
                          size_t* out_total);

/* message.zig:699-969 Message.validate over a framed message (Message.init first,
 * message.zig:341-394). Returns a capnp_packed_status code (include/capnp_packed.h):
 * 0 OK; Message.init: 8 EndOfStream, 9 InvalidSegmentCount, 10
 * SegmentCountLimitExceeded, 13 TruncatedMessage; validate: 14 EmptyMessage, 10
 * SegmentCountLimitExceeded, 13 TruncatedMessage, 15 NestingLimitExceeded, 16
 * InvalidSegmentId, 17 InvalidPointer, 18 OutOfBounds, 19 TraversalLimitExceeded, 20
 * InvalidFarPointer, 21 InvalidInlineCompositePointer, 22 ListTooLarge. *words =
 * traversal words consumed (valid when OK). */
int oracle_validate(const uint8_t* data, size_t n, uint64_t segment_count_limit, uint64_t traversal_limit_words,
                    uint64_t nesting_limit, uint64_t* words);

/* Batch drivers over independent units (same layout as the device batch ABI);
 * OpenMP over units with `threads` threads (<= 0: all). */
void oracle_pack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n,
                       uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                       int32_t* status, int threads);
void oracle_unpack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n,
                         uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                         int32_t* status, int threads);

/* packed_fast.c: the same batch drivers on a word-at-a-time port (bench.py's cpu_baseline
 * only; units it cannot take go through oracle_pack / oracle_unpack). */
void fast_pack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n, uint8_t* out, const uint64_t* out_off,
                     uint64_t* out_len, int32_t* status, int threads);
void fast_unpack_batch(const uint8_t* in, const uint64_t* in_off, uint32_t n, uint8_t* out, const uint64_t* out_off,
                       uint64_t* out_len, int32_t* status, int threads);

/* Host twin of capnp_packed_generate (include/capnp_packed.h). */
void oracle_generate(uint8_t* out, uint64_t n_units, uint64_t unit_bytes, uint64_t unit_base,
                     uint64_t seed, uint32_t zero_thresh, int threads);
uint64_t oracle_mix64(uint64_t seed, uint64_t unit, uint64_t word);

#ifdef __cplusplus
}
#endif

#endif
