/*
 * capnp_packed.h — C-ABI of the MI355X-native Cap'n Proto *packed* codec.
 *
 * This is the drop-in boundary for the reference's packed read/write surface
 * (nullstyle/capnp-zig, src/serialization/message.zig). Every entry point below
 * names the reference function it replaces. The reference functions are
 * file-private Zig functions; INTEGRATION.md shows the `extern fn` binding and the
 * three-line patch a maintainer applies to message.zig to route them here.
 *
 * Signatures use plain pointers, sizes and an opaque stream handle only.
 *
 * Codec rules are the Zig rules (NOT canonical C++ capnp): see DESIGN.md §1.
 *
 * Ownership: the caller owns every buffer. Output capacity is passed in; the
 * library never allocates caller-visible memory. A Zig caller allocates
 * `capnp_packed_encode_bound(n)` (or the size from `capnp_packed_decoded_size`)
 * and shrinks with `allocator.realloc`, which keeps Zig's exact-length free
 * contract (message.zig:144/270 `toOwnedSlice`).
 *
 * Threading: all functions are thread-safe. The single-buffer host functions
 * serialise on one internal device context. One-time device init is guarded by
 * std::call_once. Batch functions keep per-(device, caller stream) state only:
 * encode/encoded_size/decode batches put their long units (more than 4 KiB in;
 * packed units beyond the fast decoder's window) on a side stream of THAT caller
 * stream, forked from and joined back into `stream` inside the call, so ordering
 * on `stream` is as if everything ran on it and batches on different caller
 * streams never wait on each other.
 */
#ifndef CAPNP_PACKED_H
#define CAPNP_PACKED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version (INTEGRATION.md §5 lists what changed):
 *   2 (round 5): capnp_packed_framer_* and capnp_packed_set_launch_flags (added in round 4),
 *     capnp_packed_stream_contexts, CAPNP_PACKED_DECODER_WORDS; CAPNP_PACKED_DECODER_FUSED /
 *     _STREAM answer INVALID_ARGUMENT (those decoders were removed from the library in round 5,
 *     source at 869fccf), and the CPK_DECODE environment variable is gone
 *     (capnp_packed_set_decoder is the only selector). Round 6 changed no signature. */
#define CAPNP_PACKED_ABI_VERSION 2u

/* Status codes. The first four mirror the reference's error set
 * (message.zig:201 InvalidMessageSize, :105/:115/:121/:127/:137 UnexpectedEof,
 * :163/:168 Overflow, allocator OutOfMemory -> OUT_OF_SPACE because the caller
 * supplies capacity). */
enum capnp_packed_status {
    CAPNP_PACKED_OK = 0,
    CAPNP_PACKED_INVALID_MESSAGE_SIZE = 1, /* encode input length % 8 != 0 (message.zig:201) */
    CAPNP_PACKED_UNEXPECTED_EOF = 2,       /* truncated packed input (message.zig:152-191) */
    CAPNP_PACKED_OVERFLOW = 3,             /* decoded size overflows size_t (message.zig:163); unreachable for < 2^60-byte inputs */
    CAPNP_PACKED_OUT_OF_SPACE = 4,         /* output capacity too small; *out_len holds the required size */
    CAPNP_PACKED_INVALID_ARGUMENT = 5,     /* null pointer, decreasing offsets, or a misaligned word-side offset */
    CAPNP_PACKED_DEVICE_ERROR = 6,         /* HIP runtime error; see capnp_packed_last_error() */
    CAPNP_PACKED_NO_DEVICE = 7,            /* no gfx950 device / HIP code object not loadable */
    /* Reader.readPackedMessage (reader.zig:84-156) only: */
    CAPNP_PACKED_END_OF_STREAM = 8,             /* the stream ends inside the message (readByte/readNoEof) */
    CAPNP_PACKED_INVALID_SEGMENT_COUNT = 9,     /* segment count - 1 == 0xFFFFFFFF (reader.zig:123) */
    CAPNP_PACKED_SEGMENT_COUNT_LIMIT_EXCEEDED = 10, /* more than 512 segments (reader.zig:125) */
    CAPNP_PACKED_MESSAGE_TOO_LARGE = 11,        /* more than 8 Mi words (reader.zig:140) */
    CAPNP_PACKED_INVALID_PACKED_MESSAGE = 12,   /* the last record overshoots the framed length (reader.zig:151-153) */
    /* Message.init (message.zig:341-394) only: */
    CAPNP_PACKED_TRUNCATED_MESSAGE = 13,        /* header or a segment runs past the data (message.zig:353/380) */
    /* Message.validate (message.zig:699-969) only: */
    CAPNP_PACKED_EMPTY_MESSAGE = 14,            /* no segments (:700) */
    CAPNP_PACKED_NESTING_LIMIT_EXCEEDED = 15,   /* a non-null pointer past the nesting limit (:724) */
    CAPNP_PACKED_INVALID_SEGMENT_ID = 16,       /* a pointer or landing pad names a missing segment (:421/:431/:725/:761) */
    CAPNP_PACKED_INVALID_POINTER = 17,          /* pointer type 3 (capability) where data is validated (:732) */
    CAPNP_PACKED_OUT_OF_BOUNDS = 18,            /* an object runs past its segment (bounds.zig:10-13) */
    CAPNP_PACKED_TRAVERSAL_LIMIT_EXCEEDED = 19, /* more words than traversal_limit_words (:711) */
    CAPNP_PACKED_INVALID_FAR_POINTER = 20,      /* malformed double-far landing pad (:758-760, :771) */
    CAPNP_PACKED_INVALID_INLINE_COMPOSITE_POINTER = 21, /* bad inline-composite tag (:585-596, :835-845, :938) */
    CAPNP_PACKED_LIST_TOO_LARGE = 22            /* list size overflows (:945; unreachable: sizes < 2^46 words) */
};

/* Version / capability query (precedent: src/wasm/capnp_host_abi.zig:60-70). */
uint32_t capnp_packed_abi_version(void);

/* Message of the last failing call on this thread (precedent:
 * capnp_host_abi.zig:165-184 last-error). Never NULL. */
const char* capnp_packed_last_error(void);

/* Name of a status code, e.g. "UnexpectedEof" (the reference's error names). */
const char* capnp_packed_status_name(int status);

/* Upper bound on the packed size of an n-byte input: 10 * (n / 8).
 * Replaces the implicit growth of std.ArrayList in packPacked (message.zig:204-270). */
size_t capnp_packed_encode_bound(size_t n);

/* ------------------------------------------------------------------------
 * Single-buffer functions on HOST memory (one unit through the GPU).
 * ------------------------------------------------------------------------ */

/* Replaces `fn packPacked(allocator, bytes) ![]u8` (message.zig:200-271).
 * Writes the packed bytes to out[0..*out_len). On OUT_OF_SPACE, *out_len is the
 * required size and out is untouched. */
int capnp_packed_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* Replaces `fn estimateUnpackedSize(packed) !usize` (message.zig:152-191). */
int capnp_packed_decoded_size(const uint8_t* in, size_t n, size_t* out_size);

/* Replaces `fn unpackPacked(allocator, packed) ![]u8` (message.zig:88-145).
 * One host-to-device copy and one device decode into a device slot of min(cap, 8 n,
 * at least 64 KiB) bytes; if the unit needs more and cap holds it, the decode runs again
 * from the input already on the device into a slot of exactly that size. The output is
 * copied back only when the unit is OK, so errors are raised before any output byte
 * reaches `out`, as in the reference (size pass first), and out is untouched on any
 * error. On OUT_OF_SPACE, *out_len is the required size: a caller may pass a guessed
 * capacity and call again with the exact one. The device buffers grow with the largest
 * call and are given back by the next call needing a quarter of them or less (> 64 MiB). */
int capnp_packed_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* ------------------------------------------------------------------------
 * Batch functions on DEVICE memory (the hot path).
 *
 * A batch is n independent units. Unit i's input is
 *   d_in[d_in_off[i] .. d_in_off[i] + d_in_len[i])
 * and its output goes to the capacity slot
 *   d_out[d_out_off[i] .. d_out_off[i] + d_out_cap[i])
 * d_out_len[i] receives the produced (or, on OUT_OF_SPACE, required) length and
 * d_status[i] the unit's status. All arrays have n entries and live in device
 * memory; offsets/lengths are u64 bytes. Because lengths are separate arrays,
 * an encode's d_out_off/d_out_len can be passed unchanged as a decode's
 * d_in_off/d_in_len (decode straight from the capacity slots), and dense
 * streams come from capnp_packed_lengths_to_offsets.
 *
 * Word-side alignment: the unpacked side of every unit (encode input, decode
 * output) must start at a multiple of 8 bytes (INVALID_ARGUMENT otherwise); the
 * packed side may start anywhere (dense packed streams are supported).
 *
 * `stream` is a hipStream_t (NULL = default stream). Calls are asynchronous:
 * they enqueue kernels and return. The return value reports launch errors only;
 * per-unit results are in d_status / d_out_len. A unit that fails never has a byte
 * written past its out_cap, or outside its slot. Inside the slot, at every batch size,
 * the default contract is: the content of a failed decode unit's [0, out_cap) is
 * unspecified (the streaming kernels, for small units and for the words decoder's mid
 * units, may leave a prefix of its output), and likewise for an encode unit that ends
 * OUT_OF_SPACE. capnp_packed_set_all_or_nothing(1) makes every failed decode unit leave
 * its slot untouched, as unpackPacked does (message.zig:88-145 returns the error before
 * any output); or run capnp_packed_decoded_size_batch first.
 *
 * Workspace: encode / encoded_size / decode batches need a class workspace of
 * capnp_packed_batch_workspace_bytes(n) bytes (~750 B per unit + ~6 MiB: the small / mid /
 * long unit lists, the per-block class counts, the long-unit tile / window table, and
 * 704 B per unit of piece records for the indexed decoder, kept out of the caller's
 * output slots). The plain calls
 * use a queue the library keeps per caller stream (made on the first batch, grown to at
 * least twice its size on a batch larger than it holds; growing is refused with
 * DEVICE_ERROR inside a hipGraph capture). A replaced queue is freed once the stream has
 * drained, unless a capture used it: graphs that captured it stay valid, and it is kept
 * until capnp_packed_stream_release. The *_ws calls take the caller's device workspace
 * instead (256-B aligned, as hipMalloc returns; INVALID_ARGUMENT otherwise): nothing
 * of the library's is captured, and a graph of them may replay beside any work.
 * ------------------------------------------------------------------------ */

/* Batch packPacked (message.zig:200-271), one unit = one packPacked call. */
int capnp_packed_encode_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                              uint32_t n, uint8_t* d_out, const uint64_t* d_out_off,
                              const uint64_t* d_out_cap, uint64_t* d_out_len, int32_t* d_status,
                              void* stream);

/* Bytes of device workspace the *_batch_ws calls need for n units. */
size_t capnp_packed_batch_workspace_bytes(uint32_t n);

/* Free what the library keeps for a caller stream (its side stream, events and queues,
 * also queues a captured graph used). Call after the stream's work is done, before the
 * stream is destroyed, and only when no graph captured from it will replay again. The
 * next batch on the stream starts a new context. Synchronises the stream. */
int capnp_packed_stream_release(void* stream);

/* The queue the library holds for a caller stream: its size in bytes (0: none) and how
 * many replaced queues it keeps because a hipGraph capture used them. */
int capnp_packed_stream_queue_info(void* stream, size_t* bytes, uint32_t* kept);

/* How many caller streams the library holds a context for (on the current device): a leak
 * check. A framer session's own stream is released with the session (round 5). */
int capnp_packed_stream_contexts(uint32_t* count);

/* capnp_packed_encode_batch with a caller-owned device workspace of at least
 * capnp_packed_batch_workspace_bytes(n) bytes (NULL = the library's per-stream
 * queue). The workspace must not be used by another batch in flight. */
int capnp_packed_encode_batch_ws(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                 uint32_t n, uint8_t* d_out, const uint64_t* d_out_off,
                                 const uint64_t* d_out_cap, uint64_t* d_out_len, int32_t* d_status,
                                 void* d_workspace, size_t workspace_bytes, void* stream);

/* Packed sizes only (no output written): the first half of a dense encode
 * (sizes -> exclusive scan -> capnp_packed_encode_batch with dense offsets). */
int capnp_packed_encoded_size_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint64_t* d_out_len, int32_t* d_status, void* stream);

/* Batch unpackPacked (message.zig:88-145). */
int capnp_packed_decode_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                              uint32_t n, uint8_t* d_out, const uint64_t* d_out_off,
                              const uint64_t* d_out_cap, uint64_t* d_out_len, int32_t* d_status,
                              void* stream);

/* capnp_packed_decode_batch with a caller-owned device workspace (as
 * capnp_packed_encode_batch_ws). */
int capnp_packed_decode_batch_ws(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                 uint32_t n, uint8_t* d_out, const uint64_t* d_out_off,
                                 const uint64_t* d_out_cap, uint64_t* d_out_len, int32_t* d_status,
                                 void* d_workspace, size_t workspace_bytes, void* stream);

/* Batch estimateUnpackedSize (message.zig:152-191). */
int capnp_packed_decoded_size_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint64_t* d_out_len, int32_t* d_status, void* stream);

/* Batch Reader.readPackedMessage (reader.zig:84-156). Unit i is the buffered
 * packed byte stream of one reader (e.g. one connection). ONE message is decoded
 * from its front, stopping at the framed length its segment table declares; the
 * bytes after it (the next message) are not read.
 *   d_out_len[i]  framed (unpacked) bytes written to the slot
 *   d_consumed[i] packed bytes the message took: the caller advances the reader
 *                 by it and calls again for the next message
 * Per-unit errors leave d_consumed = 0 and d_out_len = 0:
 *   END_OF_STREAM (the message is incomplete: call again with more bytes),
 *   INVALID_SEGMENT_COUNT, SEGMENT_COUNT_LIMIT_EXCEEDED, MESSAGE_TOO_LARGE,
 *   INVALID_PACKED_MESSAGE (the last record overshoots the framed length).
 * OUT_OF_SPACE instead reports the framed length in d_out_len and the message's
 * packed length in d_consumed (retry with a larger slot). */
int capnp_packed_read_message_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint8_t* d_out, const uint64_t* d_out_off,
                                    const uint64_t* d_out_cap, uint64_t* d_out_len, uint64_t* d_consumed,
                                    int32_t* d_status, void* stream);

/* Connection.handleRead (src/rpc/level2/connection.zig:153-203) over n connections at
 * once, with the Framer's popFrame (src/rpc/level0/framing.zig:4-90) as
 * Reader.readPackedMessage on the device: a native host loop, HOST memory in and out.
 * Connection c's buffered bytes are in[in_off[c] .. +in_len[c]) of in[0..in_bytes).
 * One H2D of the input, then rounds of the batched reader (one unit per connection
 * that may still hold a message); each round's frames are copied D2H straight into
 * `frames`, so frame i is frames[frame_off[i] .. +frame_len[i]) of connection
 * frame_conn[i] (frames of a connection in order; *n_frames of them).
 * slot_guess[c] (in/out): the device slot for c's next frame (its last frame's size;
 *   a round that reports OUT_OF_SPACE is redone for c with the framed length).
 * consumed[c]: packed bytes of c's popped frames (the caller drops them from its buffer).
 * status[c]: END_OF_STREAM when c's bytes end inside a message or are used up (the rest
 *   waits for the next read: popFrame's null), else the reader's error that closes c
 *   (frames popped before it are still listed).
 * Returns OUT_OF_SPACE when `frames` (frames_cap bytes) or the frame table (max_frames)
 * is too small: nothing is valid then; retry with larger ones. */
int capnp_packed_frame_connections(const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                                   const uint64_t* in_len, uint32_t n, uint64_t* slot_guess, uint8_t* frames,
                                   uint64_t frames_cap, uint64_t* frame_off, uint64_t* frame_len,
                                   uint32_t* frame_conn, uint32_t max_frames, uint64_t* consumed, int32_t* status,
                                   uint32_t* n_frames);

/* Resumable framing of packed socket streams: Connection.handleRead
 * (src/rpc/level2/connection.zig:153-203) over n connections whose Framer state lives on the
 * device between reads (src/rpc/level0/framing.zig:42-90 keeps expected_total across pushes;
 * Reader.readPackedMessage, reader.zig:84-156, is one pass). A session keeps each connection's
 * unconsumed packed bytes in device memory, the current message's framed length once its
 * header is decoded, and where the walk to its end stopped: a read uploads only its new bytes
 * and the walk resumes there, so a message split over k reads is uploaded once and walked
 * once. A session is used by one thread at a time (calls serialise on it). */
typedef struct capnp_packed_framer capnp_packed_framer;
int capnp_packed_framer_create(uint32_t n_conns, capnp_packed_framer** out);
int capnp_packed_framer_destroy(capnp_packed_framer* f);
/* Append the new reads and pop every whole message. Connection c's new bytes are
 * in[in_off[c] .. +in_len[c]) of in[0..in_bytes) (in_len[c] = 0: none; in_off / in_len may be
 * NULL when in_bytes is 0). Frames as capnp_packed_frame_connections: frame i is
 * frames[frame_off[i] .. +frame_len[i]) of connection frame_conn[i], a connection's frames in
 * order. status[c] (n entries): END_OF_STREAM (its bytes end inside a message or are used up:
 * popFrame's null), or the reader's error, after which the connection's bytes are dropped (the
 * reset handleRead does, connection.zig:175-184; frames popped before it are listed).
 * OUT_OF_SPACE: `frames` or the frame table filled up; the listed frames are valid and popped,
 * the other whole messages stay buffered: call again (in_bytes = 0) to pop them.
 * One walk pass finds every whole message a connection holds (up to 64 per pass), one decode
 * pass frames them all; page-locked `in` and `frames` let the copies run at the link's rate. */
int capnp_packed_framer_read(capnp_packed_framer* f, const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                             const uint64_t* in_len, uint8_t* frames, uint64_t frames_cap, uint64_t* frame_off,
                             uint64_t* frame_len, uint32_t* frame_conn, uint32_t max_frames, int32_t* status,
                             uint32_t* n_frames);
/* capnp_packed_framer_read over the connections' own buffers (the reference keeps one
 * Framer.buffer per connection, framing.zig:6-8): connection c's new bytes are
 * in_ptr[c][0 .. in_len[c]) (in_len[c] = 0: none, in_ptr[c] may then be NULL). The library
 * gathers them into a page-locked staging buffer of the session (by byte range over up to 8
 * threads from 4 MiB up) and uploads that; no caller-side layout or pinning is needed. Frames,
 * status and OUT_OF_SPACE as capnp_packed_framer_read (call that, with in_bytes = 0, to pop the
 * rest). */
int capnp_packed_framer_readv(capnp_packed_framer* f, const uint8_t* const* in_ptr, const uint64_t* in_len,
                              uint8_t* frames, uint64_t frames_cap, uint64_t* frame_off, uint64_t* frame_len,
                              uint32_t* frame_conn, uint32_t max_frames, int32_t* status, uint32_t* n_frames);
/* Framer.reset (framing.zig:34-37) of one connection: its buffered bytes and state dropped. */
int capnp_packed_framer_reset(capnp_packed_framer* f, uint32_t conn);
/* Framer.bufferedBytes (framing.zig:30-32): packed bytes held for the connection. */
int capnp_packed_framer_buffered(capnp_packed_framer* f, uint32_t conn, uint64_t* bytes);
/* Framer.expected_total (framing.zig:10, :89): framed bytes of the connection's current message
 * once its header has been decoded, else 0. After OUT_OF_SPACE from capnp_packed_framer_read,
 * a frames buffer of the largest such size (rounded up to 8) pops that message. */
int capnp_packed_framer_expected(capnp_packed_framer* f, uint32_t conn, uint64_t* framed_bytes);
/* Bytes copied host-to-device (every read's bytes once) and moved between device regions since
 * the session was made (a connection's bytes move when its region doubles). */
int capnp_packed_framer_stats(capnp_packed_framer* f, uint64_t* uploaded, uint64_t* moved);

/* Single-buffer Reader.readPackedMessage on HOST memory: decodes the message at
 * the front of in[0..n) into out[0..*out_len); *consumed = packed bytes used.
 * On OUT_OF_SPACE, *out_len is the framed length. */
int capnp_packed_read_message(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len,
                              size_t* consumed);

/* MessageBuilder.toPackedBytes (message.zig:2175-2179 = packPacked(toBytes()),
 * toBytes 2123-2170) for n messages, packed straight from their segments: the
 * framed bytes (segment table + segments) are never materialised. Message i has
 * d_seg_count[i] segments (0 = one empty segment, as toBytes adds one) listed
 * from index d_seg_first[i] of d_seg_ptr (device addresses, 8-byte aligned) and
 * d_seg_len (bytes, multiples of 8, as a MessageBuilder's segments are). At most
 * 512 segments per message (Message.max_segment_count, message.zig:310): more,
 * or a misaligned segment, gives INVALID_ARGUMENT. Output as in
 * capnp_packed_encode_batch; d_out == NULL computes the packed sizes only. */
int capnp_packed_encode_message_batch(const uint64_t* d_seg_ptr, const uint64_t* d_seg_len,
                                      const uint32_t* d_seg_first, const uint32_t* d_seg_count, uint32_t n,
                                      uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_cap,
                                      uint64_t* d_out_len, int32_t* d_status, void* stream);

/* Message.init (message.zig:341-394) segment-table parse of n framed messages
 * d_in[d_in_off[i] .. + d_in_len[i]) (e.g. the output of a decode batch).
 * d_seg_count[i] = segments; segment j < max_segs of message i is
 * d_in[d_in_off[i] + d_seg_off[i*max_segs + j] .. + d_seg_len[i*max_segs + j]).
 * Errors per message: END_OF_STREAM (< 4 bytes), INVALID_SEGMENT_COUNT,
 * SEGMENT_COUNT_LIMIT_EXCEEDED, TRUNCATED_MESSAGE. Trailing bytes after the last
 * segment are ignored, as in the reference. */
int capnp_packed_message_init_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                    uint32_t n, uint32_t max_segs, uint32_t* d_seg_count, uint64_t* d_seg_off,
                                    uint64_t* d_seg_len, int32_t* d_status, void* stream);

/* Message.validate (message.zig:699-969, ValidationOptions :331-335) of n framed
 * messages d_in[d_in_off[i] .. + d_in_len[i]): Message.init's segment-table parse
 * (its errors: END_OF_STREAM, INVALID_SEGMENT_COUNT, SEGMENT_COUNT_LIMIT_EXCEEDED,
 * TRUNCATED_MESSAGE), then the depth-first pointer traversal with the reference's
 * limits and error order. d_status[i] = the first error the reference's recursion
 * would raise, or OK; d_words[i] (may be NULL) = traversal words consumed (OK only).
 * The reference defaults are segment_count_limit 512, traversal_limit_words 8 Mi,
 * nesting_limit 64. Any nesting_limit is accepted: up to 64 the call allocates nothing
 * and is capturable in a hipGraph; above 64, messages that need more than 64 stack frames
 * are validated by a second kernel with its frames in global memory, allocated
 * stream-ordered on `stream` (hipMallocAsync: 4n + 16 B and at most ~256 MiB of frame
 * stacks, freed stream-ordered). A nesting_limit above 2^18 is applied as 2^18 (far
 * deeper than the reference's recursive validate can go before its thread stack runs
 * out). A message of 4 GiB or more gets INVALID_ARGUMENT as its status. */
int capnp_packed_validate_batch(const uint8_t* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                uint32_t n, uint64_t segment_count_limit, uint64_t traversal_limit_words,
                                uint32_t nesting_limit, int32_t* d_status, uint64_t* d_words, void* stream);

/* Exclusive scan of n lengths into n+1 offsets (d_off[0] = base, d_off[n] =
 * base + total), on device.
 * Turns capnp_packed_*_size_batch results into dense output offsets. The
 * caller supplies device scratch of capnp_packed_scan_scratch_bytes(n) bytes
 * (no allocation inside, so the call can be captured in a hipGraph). */
size_t capnp_packed_scan_scratch_bytes(uint32_t n);
int capnp_packed_lengths_to_offsets(const uint64_t* d_len, uint32_t n, uint64_t base,
                                    uint64_t* d_off, void* d_scratch, size_t scratch_bytes,
                                    void* stream);

/* Synthetic unit generator used by the benchmark and the parity tests:
 * n units of unit_bytes each, laid out densely from d_out (unit i at
 * i*unit_bytes). Byte k of word w of global unit u = unit_base + i is
 *   h  = mix64(seed, u, w); h2 = mix64(seed ^ 0xA5A5..., u, w)
 *   b  = ((h >> 8k) & 0xFF) < zero_thresh ? 0 : 1 + (((h2 >> 8k) & 0xFF) % 255)
 * i.e. zero with probability zero_thresh/256. */
int capnp_packed_generate(uint8_t* d_out, uint64_t n_units, uint64_t unit_bytes,
                          uint64_t unit_base, uint64_t seed, uint32_t zero_thresh,
                          void* stream);

/* Decoder selection for the batch decode of mid-size units (a tuning knob, not a
 * semantic one: every decoder is bit-exact):
 *   CAPNP_PACKED_DECODER_TWO_PASS  index pass + fill pass (the packed bytes are read twice);
 *   CAPNP_PACKED_DECODER_WORDS     single read: lane per unit, one output word per step
 *                                  (round 5; a failed unit may hold a prefix
 *                                  of its output unless capnp_packed_set_all_or_nothing(1));
 *   CAPNP_PACKED_DECODER_AUTO      the library's default: the words decoder for the mid units of
 *                                  more than 1280 packed bytes into slots of at most 8 KiB when a
 *                                  batch has at least a resident grid of them (~196K units on
 *                                  MI355X), the two-pass decoder for the rest;
 *                                  all two-pass under capnp_packed_set_all_or_nothing(1).
 * The words decoder steps one output word at a time and stops a unit at its slot's capacity
 * (its size then comes from a record walk), so no unit costs it more than out_cap / 8 steps.
 * Removed in round 5 (source at 869fccf), both measured slower than the
 * two-pass decoder: CAPNP_PACKED_DECODER_FUSED (per-lane 8-state entry maps) and
 * CAPNP_PACKED_DECODER_STREAM (lane-per-unit walk by 64-B windows); the library returns
 * CAPNP_PACKED_INVALID_ARGUMENT for them.
 * Returns the previous value; applies to batches enqueued after the call (process-wide). */
enum {
    CAPNP_PACKED_DECODER_AUTO = 0,
    CAPNP_PACKED_DECODER_TWO_PASS = 1,
    CAPNP_PACKED_DECODER_FUSED = 2,
    CAPNP_PACKED_DECODER_STREAM = 3,
    CAPNP_PACKED_DECODER_WORDS = 4
};
int capnp_packed_set_decoder(int decoder);

/* All-or-nothing for small decode units too (process-wide, for batches enqueued from
 * now on; returns the previous setting, 0 or 1). Long units, and mid units the two-pass
 * decoder takes, always leave a failed unit's slot untouched (message.zig:90 raises before any
 * output). Small units (<= 512 packed bytes into <= 8-KiB slots) are by default decoded a lane
 * each in one streaming pass, and mid units the words decoder takes (see
 * capnp_packed_set_decoder) stream their output out as they go: a failed one may keep a prefix
 * of its output (never a byte past out_cap), at any batch size (the default contract above). With on != 0, small units are decoded through LDS
 * and stored only when OK, and every mid unit goes to the two-pass decoder, at a cost (C5
 * decode 0.69 -> 0.79 ms; the headline decode 2.0 -> 2.5 ms). */
int capnp_packed_set_all_or_nothing(int on);

/* Launch policy (process-wide, for batches enqueued from now on; returns the previous flags;
 * unknown bits are ignored). No result depends on it, only where the kernels run:
 *   CAPNP_PACKED_LAUNCH_LONG_INLINE      long units run after the main grid on the caller's stream
 *                                        instead of on a side stream forked from and joined into it;
 *   CAPNP_PACKED_LAUNCH_MID_SIDE_STREAM  encode and decode: mid units on a second side stream beside
 *                                        the small units' kernel (helps batches of mostly small units
 *                                        with a few mid ones; costs a fork/join
 *                                        otherwise);
 *   CAPNP_PACKED_LAUNCH_CLASS_SCAN       the class pass's scan as a kernel of its own also for
 *                                        batches of at most 1M units (by default their scatter
 *                                        kernel does it; larger batches always launch it). */
#define CAPNP_PACKED_LAUNCH_LONG_INLINE 0x1u
#define CAPNP_PACKED_LAUNCH_MID_SIDE_STREAM 0x2u
#define CAPNP_PACKED_LAUNCH_CLASS_SCAN 0x4u
uint32_t capnp_packed_set_launch_flags(uint32_t flags);

#ifdef __cplusplus
}
#endif

#endif /* CAPNP_PACKED_H */
