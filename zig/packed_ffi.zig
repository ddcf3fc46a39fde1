//! Zig binding of include/capnp_packed.h for nullstyle/capnp-zig.
//!
//! Drop this file next to src/serialization/message.zig and apply the patch in
//! INTEGRATION.md. The three wrappers below have exactly the signatures and error
//! behaviour of the file-private functions they replace:
//!   packPacked            message.zig:200-271
//!   unpackPacked          message.zig:88-145
//!   estimateUnpackedSize  message.zig:152-191
//! and `readPackedMessageBuffered` serves Reader.readPackedMessage (reader.zig:84-156)
//! for readers whose bytes are already buffered (a socket framer's read buffer).
//! Allocation follows the reference's contract: the returned slice is
//! allocator-owned with its exact length (the reference returns
//! `out.toOwnedSlice`, message.zig:144/270), so callers free it unchanged.
//!
//! Not compiled in this repo (no Zig toolchain in the build image); the C side
//! it binds is exercised by tests/test_abi.py and tests/test_gpu_parity.py.
const std = @import("std");

pub const Status = enum(c_int) {
    ok = 0,
    invalid_message_size = 1,
    unexpected_eof = 2,
    overflow = 3,
    out_of_space = 4,
    invalid_argument = 5,
    device_error = 6,
    no_device = 7,
    end_of_stream = 8,
    invalid_segment_count = 9,
    segment_count_limit_exceeded = 10,
    message_too_large = 11,
    invalid_packed_message = 12,
    truncated_message = 13,
    // Message.validate (message.zig:699-969)
    empty_message = 14,
    nesting_limit_exceeded = 15,
    invalid_segment_id = 16,
    invalid_pointer = 17,
    out_of_bounds = 18,
    traversal_limit_exceeded = 19,
    invalid_far_pointer = 20,
    invalid_inline_composite_pointer = 21,
    list_too_large = 22,
    _,
};

// ---- single-buffer host entry points -------------------------------------
extern "capnp_packed" fn capnp_packed_abi_version() u32;
extern "capnp_packed" fn capnp_packed_last_error() [*:0]const u8;
extern "capnp_packed" fn capnp_packed_encode_bound(n: usize) usize;
extern "capnp_packed" fn capnp_packed_encode(in: [*]const u8, n: usize, out: [*]u8, cap: usize, out_len: *usize) c_int;
extern "capnp_packed" fn capnp_packed_decoded_size(in: [*]const u8, n: usize, out_size: *usize) c_int;
extern "capnp_packed" fn capnp_packed_decode(in: [*]const u8, n: usize, out: [*]u8, cap: usize, out_len: *usize) c_int;
extern "capnp_packed" fn capnp_packed_read_message(in: [*]const u8, n: usize, out: [*]u8, cap: usize, out_len: *usize, consumed: *usize) c_int;
extern "capnp_packed" fn capnp_packed_frame_connections(
    in: [*]const u8, in_bytes: u64, in_off: [*]const u64, in_len: [*]const u64, n: u32,
    slot_guess: [*]u64, frames: [*]u8, frames_cap: u64, frame_off: [*]u64, frame_len: [*]u64,
    frame_conn: [*]u32, max_frames: u32, consumed: [*]u64, status: [*]i32, n_frames: *u32,
) c_int;
// Resumable framing (capnp_packed_framer_*, include/capnp_packed.h): Framer state of n
// connections kept on the device between reads (framing.zig:42-90; DESIGN.md §2.7).
pub const capnp_packed_framer = opaque {};
pub extern "capnp_packed" fn capnp_packed_framer_create(n_conns: u32, out: *?*capnp_packed_framer) c_int;
pub extern "capnp_packed" fn capnp_packed_framer_destroy(f: ?*capnp_packed_framer) c_int;
pub extern "capnp_packed" fn capnp_packed_framer_read(
    f: *capnp_packed_framer, in: ?[*]const u8, in_bytes: u64, in_off: ?[*]const u64, in_len: ?[*]const u64,
    frames: [*]u8, frames_cap: u64, frame_off: [*]u64, frame_len: [*]u64, frame_conn: [*]u32,
    max_frames: u32, status: [*]i32, n_frames: *u32,
) c_int;
// the same over each connection's own buffer (Framer.buffer, framing.zig:6-8): no layout needed
pub extern "capnp_packed" fn capnp_packed_framer_readv(
    f: *capnp_packed_framer, in_ptr: [*]const ?[*]const u8, in_len: [*]const u64,
    frames: [*]u8, frames_cap: u64, frame_off: [*]u64, frame_len: [*]u64, frame_conn: [*]u32,
    max_frames: u32, status: [*]i32, n_frames: *u32,
) c_int;
pub extern "capnp_packed" fn capnp_packed_framer_reset(f: *capnp_packed_framer, conn: u32) c_int;
pub extern "capnp_packed" fn capnp_packed_framer_buffered(f: *capnp_packed_framer, conn: u32, bytes: *u64) c_int;
pub extern "capnp_packed" fn capnp_packed_framer_expected(f: *capnp_packed_framer, conn: u32, framed_bytes: *u64) c_int;
pub extern "capnp_packed" fn capnp_packed_framer_stats(f: *capnp_packed_framer, uploaded: *u64, moved: *u64) c_int;

// ---- device batch entry points (pointers are device memory) ----------------
pub extern "capnp_packed" fn capnp_packed_encode_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out: [*]u8, d_out_off: [*]const u64, d_out_cap: [*]const u64,
    d_out_len: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
pub extern "capnp_packed" fn capnp_packed_encoded_size_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out_len: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
pub extern "capnp_packed" fn capnp_packed_decode_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out: [*]u8, d_out_off: [*]const u64, d_out_cap: [*]const u64,
    d_out_len: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
pub extern "capnp_packed" fn capnp_packed_decoded_size_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out_len: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
pub extern "capnp_packed" fn capnp_packed_read_message_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out: [*]u8, d_out_off: [*]const u64, d_out_cap: [*]const u64,
    d_out_len: [*]u64, d_consumed: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
/// MessageBuilder.toPackedBytes for n messages straight from their segment lists
/// (message.zig:2123-2179 without the toBytes copy); d_out = null: sizes only.
pub extern "capnp_packed" fn capnp_packed_encode_message_batch(
    d_seg_ptr: [*]const u64, d_seg_len: [*]const u64, d_seg_first: [*]const u32, d_seg_count: [*]const u32,
    n: u32, d_out: ?[*]u8, d_out_off: ?[*]const u64, d_out_cap: ?[*]const u64,
    d_out_len: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
/// Message.init segment-table parse (message.zig:341-394) of n framed messages.
pub extern "capnp_packed" fn capnp_packed_message_init_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32, max_segs: u32,
    d_seg_count: [*]u32, d_seg_off: [*]u64, d_seg_len: [*]u64, d_status: [*]i32, stream: ?*anyopaque,
) c_int;
/// Message.validate (message.zig:699-969) of n framed messages; ValidationOptions as
/// arguments (:331-335). d_status[i]: 0 or the first error; d_words (nullable): words consumed.
pub extern "capnp_packed" fn capnp_packed_validate_batch(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    segment_count_limit: u64, traversal_limit_words: u64, nesting_limit: u32,
    d_status: [*]i32, d_words: ?[*]u64, stream: ?*anyopaque,
) c_int;
/// Class workspace for the *_batch_ws calls (graph-safe batches with no shared state): unit
/// lists, the long-unit tile / window table and the decoder's piece records (~750 B per unit).
/// d_ws must be 256-B aligned (hipMalloc's alignment); a misaligned one is InvalidArgument.
pub extern "capnp_packed" fn capnp_packed_batch_workspace_bytes(n: u32) usize;
/// Small decode units all-or-nothing too (process-wide); returns the previous setting.
pub extern "capnp_packed" fn capnp_packed_set_all_or_nothing(on: c_int) c_int;
pub extern "capnp_packed" fn capnp_packed_set_decoder(decoder: c_int) c_int;
pub extern "capnp_packed" fn capnp_packed_set_launch_flags(flags: u32) u32;
/// Free the library's context of a caller stream (before destroying the stream).
pub extern "capnp_packed" fn capnp_packed_stream_release(stream: ?*anyopaque) c_int;
pub extern "capnp_packed" fn capnp_packed_encode_batch_ws(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out: [*]u8, d_out_off: [*]const u64, d_out_cap: [*]const u64,
    d_out_len: [*]u64, d_status: [*]i32, d_ws: ?*anyopaque, ws_bytes: usize, stream: ?*anyopaque,
) c_int;
pub extern "capnp_packed" fn capnp_packed_decode_batch_ws(
    d_in: [*]const u8, d_in_off: [*]const u64, d_in_len: [*]const u64, n: u32,
    d_out: [*]u8, d_out_off: [*]const u64, d_out_cap: [*]const u64,
    d_out_len: [*]u64, d_status: [*]i32, d_ws: ?*anyopaque, ws_bytes: usize, stream: ?*anyopaque,
) c_int;
pub extern "capnp_packed" fn capnp_packed_scan_scratch_bytes(n: u32) usize;
pub extern "capnp_packed" fn capnp_packed_lengths_to_offsets(
    d_len: [*]const u64, n: u32, base: u64, d_off: [*]u64,
    d_scratch: ?*anyopaque, scratch_bytes: usize, stream: ?*anyopaque,
) c_int;

/// Single-buffer crossover (DESIGN.md §6.1, profiles/r03_crossover.json, MI355X + EPYC 9575F
/// host, p = 0.5): one packPacked / unpackPacked call through the single-buffer C-ABI
/// (pinned staging, one H2D, kernels, D2H, sync: ~75-100 us fixed) against the Zig body's
/// algorithm on one core, caller-owned buffers on both sides.
///   pack:   the device is faster from 64 KiB (99 vs 262 us; 16 MiB: 1.6 vs 80 ms).
///   unpack: the device is faster from 64 KiB unpacked (41 KB packed: 122 vs 126 us; 164 KB
///           packed: 164 vs 631 us; 16 MiB: 2.7 vs 43 ms). The threshold below is on the
///           packed length (what unpackPacked sees): 64 KiB packed is ~100 KiB unpacked here,
///           ahead of the crossover, and zero-heavy messages (more output per packed byte)
///           favour the device further.
/// Below these sizes the patched message.zig keeps its own body; batches (many units per
/// call, capnp_packed_*_batch) are where the device pays off most.
pub const gpu_pack_min_bytes: usize = 64 * 1024;
pub const gpu_unpack_min_bytes: usize = 64 * 1024;

/// Framer dispatch (INTEGRATION.md §1.8; scripts/framer_crossover.py,
/// profiles/r05_framer_crossover.json, MI355X + EPYC 9575F host, p = 0.5): one read call of the
/// device framer session (capnp_packed_framer_readv: gather, H2D, walk, decode, D2H) against
/// the CPU reader on one core, host buffers both sides. The CPU side measured is the C oracle
/// port of the reader (oracle_read_stream: a readPackedMessage loop per connection, called
/// through ctypes; in the split case the Python driver appends each read to a bytearray), not
/// the Zig Framer itself: no Zig toolchain on the build host, so Zig parity of these CPU times
/// is unpinned.
///   N connections x 16 messages of 4 KiB framed per call: the two cross at 4 connections
///     (164 KB packed: 587 vs 611 us, 4% apart on one box); from 8 connections (328 KB) the
///     device is 2x faster (605 vs 1253 us; 4096 connections: 13.5 vs 655 ms); one connection
///     (41 KB): 518 vs 142 us. The threshold sits at the 8-connection row, with a 2x margin
///     over the crossover, not at the crossover itself.
///   one connection, a message arriving in 64 KiB reads: faster from 256 KiB framed (503 vs
///     1342 us; 16 MiB: 17.9 vs 3361 ms), since the device walk resumes across reads while the
///     CPU framer re-decodes the buffered prefix on every read.
/// A read batch goes to the device session when its new bytes reach gpu_framer_min_read_bytes,
/// or when a connection's message in progress (capnp_packed_framer_expected) is at least
/// gpu_framer_min_message_bytes; a connection moves between the two framers only while it holds
/// no partial message, so no framer state ever has to be handed over.
pub const gpu_framer_min_read_bytes: usize = 320 * 1024;
pub const gpu_framer_min_message_bytes: usize = 256 * 1024;

/// The reference's error names, plus the two the device can add. `NoDevice`
/// lets the patched message.zig fall back to its own Zig body.
pub const Error = error{
    InvalidMessageSize,
    UnexpectedEof,
    Overflow,
    OutOfMemory,
    // frameConnections: the `frames` buffer is full (grow it and call again)
    OutOfSpace,
    // a slice argument of the wrong length
    InvalidArgument,
    PackedDeviceError,
    NoDevice,
    // Reader.readPackedMessage (reader.zig:84-156)
    EndOfStream,
    InvalidSegmentCount,
    SegmentCountLimitExceeded,
    MessageTooLarge,
    InvalidPackedMessage,
    // Message.init (message.zig:341-394)
    TruncatedMessage,
    // Message.validate (message.zig:699-969)
    EmptyMessage,
    NestingLimitExceeded,
    InvalidSegmentId,
    InvalidPointer,
    OutOfBounds,
    TraversalLimitExceeded,
    InvalidFarPointer,
    InvalidInlineCompositePointer,
    ListTooLarge,
};

fn check(status: c_int) Error!void {
    return switch (@as(Status, @enumFromInt(status))) {
        .ok => {},
        .invalid_message_size => error.InvalidMessageSize,
        .unexpected_eof => error.UnexpectedEof,
        .overflow => error.Overflow,
        .out_of_space => error.OutOfMemory, // capacity is sized by us; unreachable in practice
        .no_device => error.NoDevice,
        .invalid_argument => error.InvalidArgument,
        .end_of_stream => error.EndOfStream,
        .invalid_segment_count => error.InvalidSegmentCount,
        .segment_count_limit_exceeded => error.SegmentCountLimitExceeded,
        .message_too_large => error.MessageTooLarge,
        .invalid_packed_message => error.InvalidPackedMessage,
        .truncated_message => error.TruncatedMessage,
        .empty_message => error.EmptyMessage,
        .nesting_limit_exceeded => error.NestingLimitExceeded,
        .invalid_segment_id => error.InvalidSegmentId,
        .invalid_pointer => error.InvalidPointer,
        .out_of_bounds => error.OutOfBounds,
        .traversal_limit_exceeded => error.TraversalLimitExceeded,
        .invalid_far_pointer => error.InvalidFarPointer,
        .invalid_inline_composite_pointer => error.InvalidInlineCompositePointer,
        .list_too_large => error.ListTooLarge,
        else => {
            std.log.err("capnp_packed: {s}", .{capnp_packed_last_error()});
            return error.PackedDeviceError;
        },
    };
}

/// message.zig:200 `fn packPacked(allocator, bytes) ![]u8`.
pub fn packPacked(allocator: std.mem.Allocator, bytes: []const u8) Error![]u8 {
    if (bytes.len % 8 != 0) return error.InvalidMessageSize; // message.zig:201
    const buf = try allocator.alloc(u8, capnp_packed_encode_bound(bytes.len));
    errdefer allocator.free(buf);
    var len: usize = 0;
    try check(capnp_packed_encode(bytes.ptr, bytes.len, buf.ptr, buf.len, &len));
    return allocator.realloc(buf, len);
}

/// message.zig:152 `fn estimateUnpackedSize(packed) !usize`.
pub fn estimateUnpackedSize(packed_bytes: []const u8) Error!usize {
    var size: usize = 0;
    try check(capnp_packed_decoded_size(packed_bytes.ptr, packed_bytes.len, &size));
    return size;
}

/// message.zig:88 `fn unpackPacked(allocator, packed) ![]u8`. Like the reference,
/// truncated input fails with UnexpectedEof before any output is produced. One device
/// call into a buffer of 4x the packed size; a message that expands more reports its size
/// (OUT_OF_SPACE) and is decoded again into a buffer of exactly that size.
pub fn unpackPacked(allocator: std.mem.Allocator, packed_bytes: []const u8) Error![]u8 {
    // 4x the packed size, saturating (no overflow panic in safe builds)
    var cap: usize = @max(4096, std.math.mul(usize, 4, packed_bytes.len) catch std.math.maxInt(usize));
    var attempt: u32 = 0;
    while (true) : (attempt += 1) {
        const out = try allocator.alloc(u8, cap);
        var len: usize = 0;
        const st = capnp_packed_decode(packed_bytes.ptr, packed_bytes.len, out.ptr, out.len, &len);
        if (st == @intFromEnum(Status.out_of_space) and len > cap and attempt == 0) {
            allocator.free(out);
            cap = len;
            continue;
        }
        check(st) catch |err| {
            allocator.free(out);
            return err;
        };
        // a failed shrink must not leak `out`
        return allocator.realloc(out, len) catch |err| {
            allocator.free(out);
            return err;
        };
    }
}

pub const ReadResult = struct { framed: []u8, consumed: usize };

/// reader.zig:84 `readPackedMessage(allocator, reader) ![]const u8` over bytes the
/// caller has already buffered: decodes the message at the front of `buffered`,
/// returns its framed bytes (allocator-owned, exact length) and the packed bytes it
/// took; the caller advances its buffer by `consumed`. EndOfStream means the buffer
/// holds only part of the message (read more and call again).
pub fn readPackedMessageBuffered(allocator: std.mem.Allocator, buffered: []const u8) Error!ReadResult {
    var cap: usize = @max(4096, std.math.mul(usize, 8, buffered.len) catch std.math.maxInt(usize));
    while (true) {
        const buf = try allocator.alloc(u8, cap);
        var len: usize = 0;
        var used: usize = 0;
        const st = capnp_packed_read_message(buffered.ptr, buffered.len, buf.ptr, buf.len, &len, &used);
        if (st == @intFromEnum(Status.out_of_space) and len > cap) {
            allocator.free(buf); // a zero-run heavy message: retry with its framed length
            cap = len;
            continue;
        }
        check(st) catch |err| {
            allocator.free(buf);
            return err;
        };
        const framed = allocator.realloc(buf, len) catch |err| {
            allocator.free(buf); // a failed shrink must not leak `buf`
            return err;
        };
        return .{ .framed = framed, .consumed = used };
    }
}

/// Connection.handleRead (connection.zig:153-203) over many connections in one native
/// call: `frames` receives every popped frame; frame i is
/// frames[frame_off[i]..][0..frame_len[i]] of connection frame_conn[i]. Per connection,
/// consumed[c] bytes leave its buffer and status[c] is .end_of_stream (wait for more
/// bytes) or the error that closes it. error.OutOfSpace: grow `frames` (or the table) and
/// call again. in_len, slot_guess, consumed and status must hold in_off.len entries, and
/// table.len / table.conn table.off.len entries (error.InvalidArgument otherwise: the
/// native side writes that many).
pub const FrameTable = struct { off: []u64, len: []u64, conn: []u32 };
pub fn frameConnections(
    buffered: []const u8, in_off: []const u64, in_len: []const u64, slot_guess: []u64,
    frames: []u8, table: FrameTable, consumed: []u64, status: []i32,
) Error!u32 {
    const n = in_off.len;
    if (in_len.len != n or slot_guess.len != n or consumed.len != n or status.len != n) return error.InvalidArgument;
    if (table.len.len != table.off.len or table.conn.len != table.off.len) return error.InvalidArgument;
    if (n > std.math.maxInt(u32) or table.off.len > std.math.maxInt(u32)) return error.InvalidArgument;
    var nf: u32 = 0;
    const st = capnp_packed_frame_connections(
        buffered.ptr, buffered.len, in_off.ptr, in_len.ptr, @intCast(n), slot_guess.ptr,
        frames.ptr, frames.len, table.off.ptr, table.len.ptr, table.conn.ptr, @intCast(table.off.len),
        consumed.ptr, status.ptr, &nf,
    );
    if (st == @intFromEnum(Status.out_of_space)) return error.OutOfSpace;
    try check(st);
    return nf;
}

/// ValidationOptions.nesting_limit (usize, message.zig:334) as the C-ABI's u32: the device
/// applies at most 2^18 levels anyway (capnp_packed.h), so clamping loses nothing.
pub fn nestingLimitArg(nesting_limit: usize) u32 {
    return @intCast(@min(nesting_limit, std.math.maxInt(u32)));
}

/// A validate_batch per-message status as the error Message.validate would return.
pub fn validateBatchStatus(status: i32) Error!void {
    return check(status);
}

pub fn abiVersion() u32 {
    return capnp_packed_abi_version();
}
