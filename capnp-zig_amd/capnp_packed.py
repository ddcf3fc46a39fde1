"""Host-side mirror of the reference's packed read/write surface over the C-ABI.

The reference (nullstyle/capnp-zig) exposes packing through
  MessageBuilder.toPackedBytes / writePackedTo   src/serialization/message.zig:2175-2213
  Message.initPacked                             message.zig:400-408
  Reader.initPacked                              src/serialization/reader.zig:18-23
over the file-private packPacked / unpackPacked / estimateUnpackedSize
(message.zig:88-271). This module keeps those names, argument meanings and error
names, and routes every byte through libcapnp_packed.so (HIP kernels for gfx950).
There is no CPU fallback: if the library or a gfx950 device is missing, calls
raise NoDevice / RuntimeError.

Batch functions take torch tensors that live in device memory (torch is used only
for device memory and streams): uint8 byte buffers, int64 offset/length tensors
(bit-identical to the ABI's u64), int32 status tensors.
"""
from __future__ import annotations

import ctypes
from collections import deque
import gc
import os
import struct

import numpy as np

try:  # load torch first so libcapnp_packed.so binds to the same HIP runtime instance
    import torch
except ImportError:  # pragma: no cover - the ABI still loads for symbol checks
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# CPK_LIB selects an experimental build of the same library (scripts/ diagnostics only)
LIB_PATH = os.environ.get("CPK_LIB") or os.path.join(HERE, "lib", "libcapnp_packed.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "capnp_packed.h")

OK = 0
INVALID_MESSAGE_SIZE = 1
UNEXPECTED_EOF = 2
OVERFLOW = 3
OUT_OF_SPACE = 4
INVALID_ARGUMENT = 5
DEVICE_ERROR = 6
NO_DEVICE = 7
# Reader.readPackedMessage (reader.zig:84-156)
END_OF_STREAM = 8
INVALID_SEGMENT_COUNT = 9
SEGMENT_COUNT_LIMIT_EXCEEDED = 10
MESSAGE_TOO_LARGE = 11
INVALID_PACKED_MESSAGE = 12
# Message.init (message.zig:341-394)
TRUNCATED_MESSAGE = 13
# Message.validate (message.zig:699-969)
EMPTY_MESSAGE = 14
NESTING_LIMIT_EXCEEDED = 15
INVALID_SEGMENT_ID = 16
INVALID_POINTER = 17
OUT_OF_BOUNDS = 18
TRAVERSAL_LIMIT_EXCEEDED = 19
INVALID_FAR_POINTER = 20
INVALID_INLINE_COMPOSITE_POINTER = 21
LIST_TOO_LARGE = 22


class PackedError(Exception):
    status = -1


class InvalidMessageSize(PackedError):  # message.zig:201
    status = INVALID_MESSAGE_SIZE


class UnexpectedEof(PackedError):  # message.zig:152-191
    status = UNEXPECTED_EOF


class Overflow(PackedError):  # message.zig:163
    status = OVERFLOW


class OutOfSpace(PackedError):
    status = OUT_OF_SPACE


class InvalidArgument(PackedError):
    status = INVALID_ARGUMENT


class DeviceError(PackedError):
    status = DEVICE_ERROR


class NoDevice(PackedError):
    status = NO_DEVICE


# Message.init (message.zig:341-394) and Reader.readPackedMessage (reader.zig:84-156) errors
class EndOfStream(PackedError):
    status = END_OF_STREAM


class InvalidSegmentCount(PackedError):
    status = INVALID_SEGMENT_COUNT


class SegmentCountLimitExceeded(PackedError):
    status = SEGMENT_COUNT_LIMIT_EXCEEDED


class MessageTooLarge(PackedError):  # reader.zig:140
    status = MESSAGE_TOO_LARGE


class InvalidPackedMessage(PackedError):  # reader.zig:151-153
    status = INVALID_PACKED_MESSAGE


class TruncatedMessage(PackedError):  # message.zig:353/380
    status = TRUNCATED_MESSAGE


# Message.validate (message.zig:699-969)
class EmptyMessage(PackedError):  # :700
    status = EMPTY_MESSAGE


class NestingLimitExceeded(PackedError):  # :717
    status = NESTING_LIMIT_EXCEEDED


class InvalidSegmentId(PackedError):  # :718 / :421 / :739
    status = INVALID_SEGMENT_ID


class InvalidPointer(PackedError):  # :731
    status = INVALID_POINTER


class OutOfBounds(PackedError):  # bounds.zig:10-13
    status = OUT_OF_BOUNDS


class TraversalLimitExceeded(PackedError):  # :711
    status = TRAVERSAL_LIMIT_EXCEEDED


class InvalidFarPointer(PackedError):  # :752-758
    status = INVALID_FAR_POINTER


class InvalidInlineCompositePointer(PackedError):  # :600-612 / :944
    status = INVALID_INLINE_COMPOSITE_POINTER


class ListTooLarge(PackedError):  # :949
    status = LIST_TOO_LARGE


_ERRORS = {c.status: c for c in (InvalidMessageSize, UnexpectedEof, Overflow, OutOfSpace,
                                 InvalidArgument, DeviceError, NoDevice, EndOfStream, InvalidSegmentCount,
                                 SegmentCountLimitExceeded, MessageTooLarge, InvalidPackedMessage,
                                 TruncatedMessage, EmptyMessage, NestingLimitExceeded, InvalidSegmentId,
                                 InvalidPointer, OutOfBounds, TraversalLimitExceeded, InvalidFarPointer,
                                 InvalidInlineCompositePointer, ListTooLarge)}


_lib = None
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t

# exported symbol -> (restype, argtypes)
SIGNATURES = {
    "capnp_packed_abi_version": (ctypes.c_uint32, []),
    "capnp_packed_last_error": (ctypes.c_char_p, []),
    "capnp_packed_status_name": (ctypes.c_char_p, [ctypes.c_int]),
    "capnp_packed_encode_bound": (_sz, [_sz]),
    "capnp_packed_encode": (ctypes.c_int, [_vp, _sz, _vp, _sz, ctypes.POINTER(_sz)]),
    "capnp_packed_decoded_size": (ctypes.c_int, [_vp, _sz, ctypes.POINTER(_sz)]),
    "capnp_packed_decode": (ctypes.c_int, [_vp, _sz, _vp, _sz, ctypes.POINTER(_sz)]),
    "capnp_packed_encode_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "capnp_packed_encoded_size_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp]),
    "capnp_packed_decode_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "capnp_packed_batch_workspace_bytes": (_sz, [ctypes.c_uint32]),
    "capnp_packed_encode_batch_ws": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp,
                                                    _sz, _vp]),
    "capnp_packed_decode_batch_ws": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp,
                                                    _sz, _vp]),
    "capnp_packed_decoded_size_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp]),
    "capnp_packed_read_message_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp,
                                                       _vp, _vp]),
    "capnp_packed_read_message": (ctypes.c_int, [_vp, _sz, _vp, _sz, ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    "capnp_packed_encode_message_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp,
                                                         _vp, _vp]),
    "capnp_packed_message_init_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp,
                                                       _vp, _vp, _vp]),
    "capnp_packed_validate_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint64,
                                                   ctypes.c_uint64, ctypes.c_uint32, _vp, _vp, _vp]),
    "capnp_packed_scan_scratch_bytes": (_sz, [ctypes.c_uint32]),
    "capnp_packed_lengths_to_offsets": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint64, _vp, _vp,
                                                       _sz, _vp]),
    "capnp_packed_generate": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_uint32, _vp]),
    "capnp_packed_frame_connections": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                                      ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                                      ctypes.POINTER(ctypes.c_uint32)]),
    "capnp_packed_stream_release": (ctypes.c_int, [_vp]),
    "capnp_packed_stream_contexts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32)]),
    "capnp_packed_stream_queue_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_size_t),
                                                      ctypes.POINTER(ctypes.c_uint32)]),
    "capnp_packed_set_decoder": (ctypes.c_int, [ctypes.c_int]),
    "capnp_packed_set_all_or_nothing": (ctypes.c_int, [ctypes.c_int]),
    "capnp_packed_set_launch_flags": (ctypes.c_uint32, [ctypes.c_uint32]),
    "capnp_packed_framer_create": (ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "capnp_packed_framer_destroy": (ctypes.c_int, [_vp]),
    "capnp_packed_framer_read": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp,
                                                _vp, ctypes.c_uint32, _vp, ctypes.POINTER(ctypes.c_uint32)]),
    "capnp_packed_framer_readv": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp,
                                                 ctypes.c_uint32, _vp, ctypes.POINTER(ctypes.c_uint32)]),
    "capnp_packed_framer_reset": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "capnp_packed_framer_buffered": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]),
    "capnp_packed_framer_expected": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]),
    "capnp_packed_framer_stats": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64),
                                                 ctypes.POINTER(ctypes.c_uint64)]),
}

# capnp_packed_set_decoder values (include/capnp_packed.h)
DECODERS = {"auto": 0, "twopass": 1, "fused": 2, "stream": 3, "words": 4}
# capnp_packed_set_launch_flags bits (include/capnp_packed.h)
LAUNCH_LONG_INLINE = 0x1
LAUNCH_MID_SIDE_STREAM = 0x2
LAUNCH_CLASS_SCAN = 0x4


def lib():
    """Load libcapnp_packed.so (built by `make -C capnp-zig_amd`). Fails loudly."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C capnp-zig_amd` "
                               "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        dev_build = "CPK_LIB" in os.environ  # an older dev build (same-box A/B) may lack newer entry points
        for name, (res, args) in SIGNATURES.items():
            if dev_build and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return lib().capnp_packed_last_error().decode()


def _raise(st: int, what: str = ""):
    if st == OK:
        return
    cls = _ERRORS.get(st, PackedError)
    raise cls(f"{what}: {lib().capnp_packed_status_name(st).decode()} ({last_error()})")


def _cbuf(data) -> ctypes.Array:
    b = bytes(data)
    return ctypes.create_string_buffer(b, max(1, len(b)))


# ---------------------------------------------------------------------------
# single-buffer API (host bytes in, host bytes out; one unit through the GPU)
# ---------------------------------------------------------------------------

def encode_bound(n: int) -> int:
    return lib().capnp_packed_encode_bound(n)


def pack_packed(data) -> bytes:
    """packPacked (message.zig:200-271). Raises InvalidMessageSize if len % 8."""
    data = bytes(data)
    cap = encode_bound(len(data))
    out = ctypes.create_string_buffer(max(1, cap))
    n = _sz()
    st = lib().capnp_packed_encode(_cbuf(data), len(data), out, cap, ctypes.byref(n))
    _raise(st, "packPacked")
    return out.raw[:n.value]


def estimate_unpacked_size(packed) -> int:
    """estimateUnpackedSize (message.zig:152-191)."""
    packed = bytes(packed)
    n = _sz()
    st = lib().capnp_packed_decoded_size(_cbuf(packed), len(packed), ctypes.byref(n))
    _raise(st, "estimateUnpackedSize")
    return n.value


def unpack_packed(packed, size_hint=None) -> bytes:
    """unpackPacked (message.zig:88-145). Raises UnexpectedEof on truncation.
    One device decode into a buffer of `size_hint` bytes (default 4 x the packed length):
    a message that needs more ends OUT_OF_SPACE with its size, and is decoded again into
    a buffer of exactly that size (the reference sizes first, message.zig:90)."""
    packed = bytes(packed)
    cap = max(4096, 4 * len(packed)) if size_hint is None else int(size_hint)
    for _ in range(2):
        out = ctypes.create_string_buffer(max(1, cap))
        n = _sz()
        st = lib().capnp_packed_decode(_cbuf(packed), len(packed), out, cap, ctypes.byref(n))
        if st == OUT_OF_SPACE and n.value > cap:
            cap = n.value
            continue
        _raise(st, "unpackPacked")
        return out.raw[:n.value]
    _raise(st, "unpackPacked")


# ---------------------------------------------------------------------------
# framing mirror: MessageBuilder / Message / Reader (packed entry points only)
# ---------------------------------------------------------------------------

MAX_SEGMENT_COUNT = 512  # message.zig:310


def frame_segments(segments) -> bytes:
    """MessageBuilder.toBytes (message.zig:2123-2170): segment table + segments."""
    segs = [bytes(s) for s in segments] or [b""]
    n = len(segs)
    for s in segs:
        if len(s) % 8:
            raise InvalidMessageSize("segment length is not a multiple of 8")
    hdr = struct.pack("<I", n - 1) + b"".join(struct.pack("<I", len(s) // 8) for s in segs)
    if n % 2 == 0:
        hdr += b"\x00\x00\x00\x00"
    return hdr + b"".join(segs)


class MessageBuilder:
    """Segment-level mirror of MessageBuilder (message.zig:1643). Only the
    serialization surface is mirrored; struct/list building is out of scope."""

    def __init__(self):
        self.segments: list[bytearray] = []

    def create_segment(self, data=b"") -> int:
        self.segments.append(bytearray(data))
        return len(self.segments) - 1

    def to_bytes(self) -> bytes:
        if not self.segments:
            self.create_segment()
        return frame_segments(self.segments)

    def to_packed_bytes(self) -> bytes:
        """message.zig:2175-2179: packPacked(toBytes())."""
        return pack_packed(self.to_bytes())

    def write_to(self, writer) -> None:
        writer.write(self.to_bytes())

    def write_packed_to(self, writer) -> None:
        """message.zig:2209-2213."""
        writer.write(self.to_packed_bytes())


class Message:
    """Mirror of Message (message.zig:309-418): segment views over backing data."""

    def __init__(self, segments, backing_data):
        self.segments = segments
        self.backing_data = backing_data

    @classmethod
    def init(cls, data) -> "Message":
        """message.zig:341-394 segment-table parse; borrows `data`."""
        mv = memoryview(bytes(data) if not isinstance(data, (bytes, bytearray, memoryview)) else data)
        if len(mv) < 4:
            raise EndOfStream()
        (minus_one,) = struct.unpack_from("<I", mv, 0)
        if minus_one == 0xFFFFFFFF:
            raise InvalidSegmentCount()
        count = minus_one + 1
        if count > MAX_SEGMENT_COUNT:
            raise SegmentCountLimitExceeded()
        header_bytes = (1 + count + (1 if count % 2 == 0 else 0)) * 4
        if header_bytes > len(mv):
            raise TruncatedMessage()
        sizes = struct.unpack_from(f"<{count}I", mv, 4)
        off = header_bytes
        segs = []
        for sw in sizes:
            end = off + 8 * sw
            if end > len(mv):
                raise TruncatedMessage()
            segs.append(mv[off:end])
            off = end
        return cls(segs, None)

    @classmethod
    def init_packed(cls, packed) -> "Message":
        """message.zig:400-408: unpackPacked then Message.init; owns the buffer."""
        unpacked = unpack_packed(packed)
        msg = cls.init(unpacked)
        msg.backing_data = unpacked
        return msg

    def validate(self, segment_count_limit=None, traversal_limit_words=None, nesting_limit=None,
                 device="cuda") -> int:
        """message.zig:699-969 Message.validate(options), run by validate_batch on the
        device over this message's segments (re-framed: header + segments, the bytes
        Message.init parsed). Raises the reference's error; returns the traversal words
        consumed. Arguments left None take ValidationOptions' defaults (:331-335).
        An empty segment list raises EmptyMessage (:700), as after deinit(). Segments are
        whole words when they come from Message.init / init_packed; a hand-built segment
        whose length is not a multiple of 8 cannot be framed and raises InvalidMessageSize."""
        if len(self.segments) == 0:
            raise EmptyMessage("Message.validate: no segments")
        framed = np.frombuffer(frame_segments(self.segments), dtype=np.uint8)
        d_in = torch.from_numpy(framed.copy()).to(device)
        off = torch.zeros(1, dtype=torch.int64, device=device)
        ln = torch.full((1,), framed.size, dtype=torch.int64, device=device)
        st = torch.full((1,), -1, dtype=torch.int32, device=device)
        words = torch.zeros(1, dtype=torch.int64, device=device)
        validate_batch(d_in, off, ln, st, words,
                       DEFAULT_SEGMENT_COUNT_LIMIT if segment_count_limit is None else segment_count_limit,
                       DEFAULT_TRAVERSAL_LIMIT_WORDS if traversal_limit_words is None else traversal_limit_words,
                       DEFAULT_NESTING_LIMIT if nesting_limit is None else nesting_limit)
        _raise(int(st.item()), "Message.validate")
        return int(words.item())

    def deinit(self) -> None:
        self.segments = []
        self.backing_data = None


class Reader:
    """Mirror of Reader.init / Reader.initPacked (reader.zig:11-23)."""

    def __init__(self, msg: Message):
        self.msg = msg

    @classmethod
    def init(cls, data) -> "Reader":
        return cls(Message.init(data))

    @classmethod
    def init_packed(cls, data) -> "Reader":
        return cls(Message.init_packed(data))

    @staticmethod
    def read_packed_message(reader) -> bytes:
        """Reader.readPackedMessage (reader.zig:84-156): decode the packed message at
        the front of `reader` (bytes-like, or a binary file object with read/seek)
        and return its framed bytes, stopping at the length its segment table
        declares. A file object is left just past the message; on an error it is
        left where it was."""
        if hasattr(reader, "read"):
            start = reader.tell()
            data = reader.read()
            try:
                framed, used = read_packed_message_bytes(data)
            except PackedError:
                reader.seek(start)
                raise
            reader.seek(start + used)
            return framed
        return read_packed_message_bytes(reader)[0]


def read_packed_message_bytes(data) -> tuple:
    """(framed bytes, packed bytes consumed) of the message at the front of `data`
    (reader.zig:84-156), through the single-buffer C-ABI entry point."""
    data = bytes(data)
    src = _cbuf(data)
    cap = max(4096, 8 * len(data))
    for _ in range(2):  # a zero-run heavy message can expand past the first guess
        out = ctypes.create_string_buffer(cap)
        n, used = _sz(), _sz()
        st = lib().capnp_packed_read_message(src, len(data), out, cap, ctypes.byref(n), ctypes.byref(used))
        if st == OUT_OF_SPACE and n.value > cap:
            cap = n.value
            continue
        _raise(st, "readPackedMessage")
        return out.raw[:n.value], used.value
    raise OutOfSpace("readPackedMessage: framed length grew between calls")


# ---------------------------------------------------------------------------
# Framing for packed byte streams
# ---------------------------------------------------------------------------

_PIN_MIN = 1 << 20


def _host_bytes(nbytes: int, pin: bool = True) -> np.ndarray:
    """A host byte buffer for a framer call. With `pin`, from 1 MiB up it is page-locked memory
    from torch's caching host allocator: the session's H2D / D2H copies then run at the link's
    DMA rate instead of through the runtime's pageable staging, and a freed buffer (its last
    frame view dropped) goes back to torch's cache for the next read."""
    if pin and nbytes >= _PIN_MIN and torch is not None and torch.cuda.is_available():
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()
    return np.empty(max(nbytes, 1), dtype=np.uint8)


class FramerSession:
    """A capnp_packed_framer: the Framer state of n connections kept on the device between
    reads (include/capnp_packed.h). Each connection's unconsumed packed bytes
    stay in device memory and the walk to the current message's end resumes where the last
    read left it, so a message split over k reads is uploaded once and walked once."""

    def __init__(self, n_conns: int):
        h = _vp()
        _raise(lib().capnp_packed_framer_create(int(n_conns), ctypes.byref(h)), "framer_create")
        self.handle, self.n = h, int(n_conns)

    def close(self):
        if getattr(self, "handle", None):
            lib().capnp_packed_framer_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def read(self, reads: dict):
        """Append `reads` ({connection: bytes}) and pop every whole message. Returns
        (frames, status): frames[c] lists connection c's frames in order (read-only
        memoryviews of the call's frame buffers), status an int32 array: END_OF_STREAM, or the
        reader's error after which the connection's bytes were dropped."""
        gc_on = gc.isenabled()
        gc.disable()  # no cycles among the views; the collector's passes cost more
        try:
            return self._read(reads)
        finally:
            if gc_on:
                gc.enable()

    def assemble(self, reads: dict):
        """The connections' new bytes as one host buffer (page-locked from 1 MiB up) with
        per-connection offsets and lengths: the input of read_raw."""
        n = self.n
        lens = np.zeros(n, dtype=np.uint64)
        for c, d in reads.items():
            lens[c] = len(d)
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(lens)[:-1]
        host = _host_bytes(int(lens.sum()))
        for c, d in reads.items():
            if len(d):
                host[int(off[c]):int(off[c]) + len(d)] = np.frombuffer(d, dtype=np.uint8)
        return host, off, lens

    def read_raw(self, host, off, lens):
        """capnp_packed_framer_read over an assembled input (a server that receives into one
        buffer skips assemble()). Returns (parts, status): parts lists (buf, f_off, f_len,
        f_conn) per native call, frame i of a part being buf[f_off[i]:f_off[i] + f_len[i]] of
        connection f_conn[i], a connection's frames in order over the parts; status as read()."""
        total = int(lens.sum())

        def first(*out):
            return lib().capnp_packed_framer_read(self.handle, host.ctypes.data, total, off.ctypes.data,
                                                  lens.ctypes.data, *out)
        return self._pop(first, total)

    def readv_raw(self, reads: dict):
        """read_raw over the connections' own bytes objects (capnp_packed_framer_readv: the
        library gathers them into its page-locked staging, no host-side layout)."""
        n = self.n
        ptrs = (ctypes.c_char_p * n)()
        lens = np.zeros(n, dtype=np.uint64)
        keep = []
        for c, d in reads.items():
            if len(d):
                d = d if isinstance(d, bytes) else bytes(d)
                keep.append(d)  # alive through the call
                ptrs[c] = d
                lens[c] = len(d)
        total = int(lens.sum())

        def first(*out):
            return lib().capnp_packed_framer_readv(self.handle, ptrs, lens.ctypes.data, *out)
        return self._pop(first, total)

    def _pop(self, first_call, total: int):
        n = self.n
        status = np.zeros(n, dtype=np.int32)
        parts = []
        # frames of 2x the read's bytes: the buffer runs out only for messages packed below
        # half their size, and then the loop below pops the rest into a larger one
        cap, max_frames = max(1 << 16, 2 * total + (1 << 16)), max(1024, total // 2 + 64)
        first = True
        while True:
            # a retry's buffer is sized for one large message: pageable, as pinning it fresh
            # costs more than the runtime's staged copy of it
            buf = _host_bytes(cap, pin=first)
            f_off = np.empty(max_frames, dtype=np.uint64)
            f_len = np.empty(max_frames, dtype=np.uint64)
            f_conn = np.empty(max_frames, dtype=np.uint32)
            st_call = np.zeros(n, dtype=np.int32)
            nf = ctypes.c_uint32(0)
            out = (buf.ctypes.data, cap, f_off.ctypes.data, f_len.ctypes.data, f_conn.ctypes.data, max_frames,
                   st_call.ctypes.data, ctypes.byref(nf))
            if first:
                rc = first_call(*out)
            else:  # later calls pop what is held, no new bytes
                rc = lib().capnp_packed_framer_read(self.handle, None, 0, None, None, *out)
            if rc not in (OK, OUT_OF_SPACE):
                try:
                    _raise(rc, "framer_read")
                except PackedError as exc:
                    # the session already advanced past the frames of earlier calls of this read:
                    # hand them over with the error instead of losing them (exc.partial, as read_raw
                    # returns them: (parts, status))
                    status[status == 0] = END_OF_STREAM
                    exc.partial = (parts, status)
                    raise
            first = False
            err = st_call != END_OF_STREAM
            status[err] = st_call[err]
            k = nf.value
            if k:
                parts.append((buf, f_off[:k], f_len[:k], f_conn[:k]))
            if rc == OK:
                break
            # frames or the table filled up: pop the rest into larger ones; a buffer of the
            # largest known framed length pops at least that message
            big = max((self.expected(c) for c in range(n)), default=0)
            cap = max(cap * 2 if k == 0 else cap, (big + 7) // 8 * 8 + 64)
            max_frames *= 2
        status[status == 0] = END_OF_STREAM
        return parts, status

    def _read(self, reads: dict):
        try:
            parts, status = self.readv_raw(reads)
        except PackedError as exc:
            if hasattr(exc, "partial"):  # frames popped before the failing call: exc.frames
                exc.frames = self._group(*exc.partial)[0]
            raise
        return self._group(parts, status)

    @staticmethod
    def _group(parts, status):
        frames = {}
        for buf, f_off, f_len, f_conn in parts:
            # a connection's frames are in order within a call: group them by a stable sort
            view = memoryview(buf).toreadonly()
            if len(f_conn) > 1 and bool((f_conn[1:] < f_conn[:-1]).any()):  # a later pass's frames
                order = np.argsort(f_conn, kind="stable")
                conn_s, fo, fl = f_conn[order], f_off[order], f_len[order]
            else:  # one walk pass: already grouped by connection, in order
                conn_s, fo, fl = f_conn, f_off, f_len
            fo_l, fe_l = fo.tolist(), (fo + fl).tolist()
            cuts = (np.flatnonzero(np.diff(conn_s)) + 1).tolist()
            starts = [0] + cuts
            for c, a, b in zip(conn_s[starts].tolist(), starts, cuts + [len(conn_s)]):
                frames.setdefault(c, []).extend(map(view.__getitem__, map(slice, fo_l[a:b], fe_l[a:b])))
        return frames, status

    def buffered(self, c: int) -> int:
        b = ctypes.c_uint64()
        _raise(lib().capnp_packed_framer_buffered(self.handle, int(c), ctypes.byref(b)), "framer_buffered")
        return b.value

    def expected(self, c: int) -> int:
        """Framer.expected_total (framing.zig:10): framed bytes of connection c's current
        message once its header is decoded, else 0."""
        b = ctypes.c_uint64()
        _raise(lib().capnp_packed_framer_expected(self.handle, int(c), ctypes.byref(b)), "framer_expected")
        return b.value

    def reset(self, c: int) -> None:
        _raise(lib().capnp_packed_framer_reset(self.handle, int(c)), "framer_reset")

    def stats(self) -> dict:
        up, mv = ctypes.c_uint64(), ctypes.c_uint64()
        _raise(lib().capnp_packed_framer_stats(self.handle, ctypes.byref(up), ctypes.byref(mv)), "framer_stats")
        return {"uploaded_bytes": up.value, "moved_bytes": mv.value}


class PackedFramer:
    """The RPC `Framer` (src/rpc/level0/framing.zig:4-90) for a PACKED byte stream.
    It has the same surface: push / buffered_bytes / reset / pop_frame.
    - push() appends a socket read.
    - pop_frame() returns the framed (unpacked) bytes of the next whole message, or None
      while the buffered bytes do not hold one yet (the reader's EndOfStream).
    - pop_frame() raises the reader's other errors (reader.zig:84-156). The caller then
      reset()s, as Connection.handleRead does (level2/connection.zig:175-184).
    - A message's end is only known by decoding its packed records, so the buffered bytes
      live on the device (a one-connection FramerSession): a push's bytes are uploaded once,
      and the walk to the message end resumes where the previous pop left it.
    - PackedConnections does this for many connections at once."""

    max_frame_words = 8 * 1024 * 1024  # framing.zig:5 / reader.zig:6
    max_segment_count = MAX_SEGMENT_COUNT

    def __init__(self):
        self.session = FramerSession(1)
        self.pending = []      # pushed bytes not yet handed to the session
        self.ready = deque()   # frames popped from the device (then the error that ended them)
        self.error = None      # the framing error once raised: raised again until reset()

    def push(self, data) -> None:
        if len(data):
            self.pending.append(bytes(data))

    def buffered_bytes(self) -> int:
        """Framer.bufferedBytes (framing.zig:30-32): pushed bytes not yet framed. One difference:
        pop_frame takes every whole message off the device at once, and the packed bytes of the
        frames it holds for later pop_frame calls are no longer counted (the device does not
        report each frame's packed length)."""
        return self.session.buffered(0) + sum(len(d) for d in self.pending)

    def reset(self) -> None:
        self.session.reset(0)
        self.pending.clear()
        self.ready.clear()
        self.error = None

    def pop_frame(self):
        if self.error is not None:  # framing.zig: the corrupt bytes keep failing until reset
            raise self.error
        if not self.ready and self.pending:
            data = b"".join(self.pending)
            self.pending.clear()
            frames, status = self.session.read({0: data})
            self.ready.extend(bytes(f) for f in frames.get(0, []))
            if int(status[0]) != END_OF_STREAM:
                rs = int(status[0])
                self.ready.append(_ERRORS.get(rs, DeviceError)(
                    f"readPackedMessage: {lib().capnp_packed_status_name(rs).decode()}"))
        if not self.ready:
            return None
        v = self.ready.popleft()
        if isinstance(v, Exception):
            self.error = v
            raise v
        return v


class _ConnView:
    """A PackedConnections connection's framer surface (bufferedBytes / reset)."""

    def __init__(self, session, c):
        self._s, self._c = session, c

    def buffered_bytes(self) -> int:
        return self._s.buffered(self._c)

    def reset(self) -> None:
        self._s.reset(self._c)


class PackedConnections:
    """Connection.handleRead (src/rpc/level2/connection.zig:153-203) over many
    connections at once, on one FramerSession: every connection's Framer state (its
    unconsumed packed bytes, the current message's framed length, where the walk to its end
    stopped) stays on the device between reads.
    - handle_read(reads) uploads only the new bytes and pops every whole message in one
      native call (capnp_packed_framer_read).
    - Per connection, the result is the list of frames popped (in order), or a PackedError.
    - On the error the connection's framer is reset and the connection is closed for
      further reads, as handleRead does (175-184). Frames popped before the error are
      dropped with it; handleRead would already have delivered them, so
      `frames_before_error` keeps them.
    - A connection whose bytes end inside a message keeps them for its next read (the
      reader's EndOfStream = popFrame's null), and its walk resumes there."""

    def __init__(self, n_conns: int, device="cuda"):
        self.session = FramerSession(n_conns)
        self.framers = [_ConnView(self.session, c) for c in range(n_conns)]
        self.closed = [False] * n_conns
        self.frames_before_error = {}
        self.device = torch.device(device)

    def handle_read(self, reads: dict) -> dict:
        """One native call: the connections' new bytes go to the device once, every whole
        message is popped, and the frames come back as read-only memoryviews of the call's
        frame buffer (no per-frame copy; the buffer lives as long as its frames)."""
        gc_on = gc.isenabled()
        gc.disable()  # the result's lists and views hold no cycles
        try:
            return self._handle_read(reads)
        finally:
            if gc_on:
                gc.enable()

    def _handle_read(self, reads: dict) -> dict:
        live = {c: d for c, d in reads.items() if not self.closed[c] and len(d)}
        frames, status = self.session.read(live)
        result = {c: [] for c in live}
        result.update(frames)
        for c in np.nonzero(status != END_OF_STREAM)[0].tolist():
            rs = int(status[c])
            self.frames_before_error[c] = result.get(c, [])
            result[c] = _ERRORS.get(rs, DeviceError)(f"readPackedMessage: {lib().capnp_packed_status_name(rs).decode()}")
            self.closed[c] = True
        return result


# ---------------------------------------------------------------------------
# device-resident batch API (torch tensors in HBM)
# ---------------------------------------------------------------------------

def set_decoder(name: str) -> str:
    """Select the mid-unit batch decoder ("auto", "twopass", "words"; "fused" and "stream" were
    removed in round 5 and raise) for batches enqueued from now on; returns the previous
    setting's name. Every one is bit-exact."""
    prev = lib().capnp_packed_set_decoder(DECODERS[name])
    if prev < 0 or prev not in DECODERS.values():
        _raise(prev, "set_decoder")
    return {v: k for k, v in DECODERS.items()}[prev]


def decoder_available(name: str) -> bool:
    """Whether this build has the decoder: "auto", "twopass" and "words"; not "fused" and
    "stream" (removed in round 5)."""
    L = lib()
    prev = L.capnp_packed_set_decoder(DECODERS[name])
    if prev not in DECODERS.values():
        return False
    L.capnp_packed_set_decoder(prev)
    return True


def set_all_or_nothing(on: bool) -> bool:
    """Small decode units all-or-nothing too (capnp_packed_set_all_or_nothing); returns the
    previous setting."""
    return bool(lib().capnp_packed_set_all_or_nothing(1 if on else 0))


def set_launch_flags(flags: int) -> int:
    """Launch policy bits (capnp_packed_set_launch_flags: LAUNCH_LONG_INLINE,
    LAUNCH_MID_SIDE_STREAM, LAUNCH_CLASS_SCAN); returns the previous flags. No result depends on them."""
    return int(lib().capnp_packed_set_launch_flags(int(flags)))


class launch_flags:
    """Context manager: `with launch_flags(LAUNCH_LONG_INLINE): ...` restores the flags after."""

    def __init__(self, flags: int):
        self.flags, self.prev = flags, None

    def __enter__(self):
        self.prev = set_launch_flags(self.flags)
        return self

    def __exit__(self, *exc):
        set_launch_flags(self.prev)
        return False


class decoder:
    """Context manager: `with decoder("words"): ...` restores the previous decoder after."""

    def __init__(self, name: str):
        self.name, self.prev = name, None

    def __enter__(self):
        self.prev = set_decoder(self.name)
        return self

    def __exit__(self, *exc):
        set_decoder(self.prev)
        return False


def stream_release(stream=None) -> None:
    """Free the library's context of a stream (side stream, events, queues); see
    capnp_packed_stream_release. Synchronises the stream."""
    _raise(lib().capnp_packed_stream_release(_stream(stream)), "stream_release")


def stream_queue_info(stream=None):
    """(bytes of the stream's queue, replaced queues kept for captured graphs)."""
    b, k = ctypes.c_size_t(), ctypes.c_uint32()
    _raise(lib().capnp_packed_stream_queue_info(_stream(stream), ctypes.byref(b), ctypes.byref(k)),
           "stream_queue_info")
    return b.value, k.value


def stream_contexts() -> int:
    """How many caller streams the library holds a context for (capnp_packed_stream_contexts)."""
    k = ctypes.c_uint32()
    _raise(lib().capnp_packed_stream_contexts(ctypes.byref(k)), "stream_contexts")
    return k.value


def _ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def _stream(stream) -> int:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def _units(in_off, *per_unit) -> int:
    """Unit count of a batch (in_off's length); every per-unit tensor must hold at
    least that many entries (the kernels index them by unit)."""
    n = in_off.numel()
    for t in per_unit:
        if t is not None and t.numel() < n:
            raise InvalidArgument(f"per-unit tensor has {t.numel()} entries for {n} units")
    return n


def workspace(n_units: int, device="cuda"):
    """Device workspace for the *_batch_ws calls (capnp_packed_batch_workspace_bytes):
    a batch that uses its own workspace shares no library state, so a captured
    hipGraph of it may replay beside any other work."""
    nbytes = lib().capnp_packed_batch_workspace_bytes(n_units)
    return torch.empty((nbytes + 7) // 8, dtype=torch.int64, device=device)


def _ws(ws):
    return (0, 0) if ws is None else (ws.data_ptr(), ws.numel() * ws.element_size())


def encode_batch(d_in, in_off, in_len, d_out, out_off, out_cap, out_len, status, stream=None, ws=None) -> None:
    """Batch packPacked: unit i = d_in[in_off[i] : in_off[i]+in_len[i]] -> slot
    d_out[out_off[i] : out_off[i]+out_cap[i]]; out_len[i], status[i] per unit.
    ws: optional workspace() tensor (capnp_packed_encode_batch_ws)."""
    n = _units(in_off, in_len, out_off, out_cap, out_len, status)
    if ws is None:
        _raise(lib().capnp_packed_encode_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(d_out),
                                               _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(status),
                                               _stream(stream)), "encode_batch")
    else:
        _raise(lib().capnp_packed_encode_batch_ws(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(d_out),
                                                  _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(status),
                                                  *_ws(ws), _stream(stream)), "encode_batch_ws")


def encoded_size_batch(d_in, in_off, in_len, out_len, status, stream=None) -> None:
    n = _units(in_off, in_len, out_len, status)
    _raise(lib().capnp_packed_encoded_size_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(out_len),
                                                 _ptr(status), _stream(stream)), "encoded_size_batch")


def decode_batch(d_in, in_off, in_len, d_out, out_off, out_cap, out_len, status, stream=None, ws=None) -> None:
    """Batch unpackPacked: unit i = d_in[in_off[i] : in_off[i]+in_len[i]] -> slot
    d_out[out_off[i] : out_off[i]+out_cap[i]]; out_len[i], status[i] per unit.
    ws: optional workspace() tensor (capnp_packed_decode_batch_ws)."""
    n = _units(in_off, in_len, out_off, out_cap, out_len, status)
    if ws is None:
        _raise(lib().capnp_packed_decode_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(d_out),
                                               _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(status),
                                               _stream(stream)), "decode_batch")
    else:
        _raise(lib().capnp_packed_decode_batch_ws(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(d_out),
                                                  _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(status),
                                                  *_ws(ws), _stream(stream)), "decode_batch_ws")


def decoded_size_batch(d_in, in_off, in_len, out_len, status, stream=None) -> None:
    n = _units(in_off, in_len, out_len, status)
    _raise(lib().capnp_packed_decoded_size_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(out_len),
                                                 _ptr(status), _stream(stream)), "decoded_size_batch")


def read_message_batch(d_in, in_off, in_len, d_out, out_off, out_cap, out_len, consumed, status,
                       stream=None) -> None:
    """Batch Reader.readPackedMessage (reader.zig:84-156): one message from the front
    of each unit (a reader's buffered packed stream) -> its slot; consumed[i] =
    packed bytes the message took (0 on error), out_len[i] = framed bytes."""
    n = _units(in_off, in_len, out_off, out_cap, out_len, consumed, status)
    _raise(lib().capnp_packed_read_message_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, _ptr(d_out),
                                                 _ptr(out_off), _ptr(out_cap), _ptr(out_len), _ptr(consumed),
                                                 _ptr(status), _stream(stream)), "read_message_batch")


def encode_message_batch(seg_ptr, seg_len, seg_first, seg_count, d_out, out_off, out_cap, out_len, status,
                         stream=None) -> None:
    """MessageBuilder.toPackedBytes (message.zig:2123-2179) for a batch of messages,
    packed straight from their segments. seg_ptr / seg_len: int64 tensors of segment
    device addresses and byte lengths; seg_first / seg_count: int32 tensors, one
    entry per message. d_out None = packed sizes only."""
    n = _units(seg_first, seg_count, out_len, status)
    if d_out is not None:
        _units(seg_first, out_off, out_cap)
    _raise(lib().capnp_packed_encode_message_batch(_ptr(seg_ptr), _ptr(seg_len), _ptr(seg_first), _ptr(seg_count),
                                                   n, _ptr(d_out), _ptr(out_off), _ptr(out_cap), _ptr(out_len),
                                                   _ptr(status), _stream(stream)), "encode_message_batch")


def message_init_batch(d_in, in_off, in_len, max_segs, seg_count, seg_off, seg_len, status, stream=None) -> None:
    """Message.init (message.zig:341-394) segment tables of a batch of framed messages:
    seg_count[i] (int32), seg_off / seg_len rows of max_segs entries (int64)."""
    n = _units(in_off, in_len, seg_count, status)
    if max_segs and (seg_off.numel() < n * max_segs or seg_len.numel() < n * max_segs):
        raise InvalidArgument("segment tables need n * max_segs entries")
    _raise(lib().capnp_packed_message_init_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, max_segs,
                                                 _ptr(seg_count), _ptr(seg_off), _ptr(seg_len), _ptr(status),
                                                 _stream(stream)), "message_init_batch")


# Message.ValidationOptions defaults (message.zig:331-335)
DEFAULT_SEGMENT_COUNT_LIMIT = MAX_SEGMENT_COUNT
DEFAULT_TRAVERSAL_LIMIT_WORDS = 8 * 1024 * 1024
DEFAULT_NESTING_LIMIT = 64


def validate_batch(d_in, in_off, in_len, status, words=None, segment_count_limit=DEFAULT_SEGMENT_COUNT_LIMIT,
                   traversal_limit_words=DEFAULT_TRAVERSAL_LIMIT_WORDS, nesting_limit=DEFAULT_NESTING_LIMIT,
                   stream=None) -> None:
    """Message.validate (message.zig:699-969) of a batch of framed messages (the bytes
    Message.init takes): status[i] = 0 or the reference's first error for message i;
    words[i] (optional int64) = traversal words the walk consumed (0 on error).
    Any nesting limit is accepted; the device applies at most 2^18 (the C-ABI takes a u32,
    so larger values are clamped here first)."""
    n = _units(in_off, in_len, status, words)
    nesting_limit = min(int(nesting_limit), 0xFFFFFFFF)
    _raise(lib().capnp_packed_validate_batch(_ptr(d_in), _ptr(in_off), _ptr(in_len), n, segment_count_limit,
                                             traversal_limit_words, nesting_limit, _ptr(status), _ptr(words),
                                             _stream(stream)), "validate_batch")


def lengths_to_offsets(lengths, base: int = 0, out=None, stream=None):
    """Exclusive scan of lengths -> n+1 offsets (dense output layout), on device."""
    n = lengths.numel()
    if out is None:
        out = torch.empty(n + 1, dtype=torch.int64, device=lengths.device)
    nbytes = lib().capnp_packed_scan_scratch_bytes(n)
    scratch = torch.empty((nbytes + 7) // 8, dtype=torch.int64, device=lengths.device)
    _raise(lib().capnp_packed_lengths_to_offsets(_ptr(lengths), n, base, _ptr(out), _ptr(scratch), nbytes,
                                                 _stream(stream)), "lengths_to_offsets")
    return out


def generate(n_units: int, unit_bytes: int, seed: int, zero_thresh: int, unit_base: int = 0,
             out=None, device="cuda", stream=None):
    """Device-side synthetic units; twin of the oracle generator."""
    if out is None:
        out = torch.empty(n_units * unit_bytes, dtype=torch.uint8, device=device)
    _raise(lib().capnp_packed_generate(_ptr(out), n_units, unit_bytes, unit_base, seed, zero_thresh,
                                       _stream(stream)), "generate")
    return out


def uniform_layout(n_units: int, unit_bytes: int, device="cuda"):
    """(offsets, lengths) of n equal units laid out densely; also the capacity-slot
    layout of an encode output (unit_bytes = encode_bound(unit size))."""
    off = torch.arange(0, n_units * unit_bytes, unit_bytes, dtype=torch.int64, device=device)
    ln = torch.full((n_units,), unit_bytes, dtype=torch.int64, device=device)
    return off, ln
