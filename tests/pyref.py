"""Independent pure-Python restatement of the Zig packed codec (test-only).

Written from the rule statement, not from the C oracle,
so that the two restatements cross-check each other on small inputs:

  encoder  nullstyle/capnp-zig src/serialization/message.zig:200-271
  decoder  message.zig:88-145, size pass message.zig:152-191
  stream   src/serialization/reader.zig:84-156

Errors are raised as exceptions named after the reference's Zig errors.
"""


class InvalidMessageSize(Exception):
    pass


class UnexpectedEof(Exception):
    pass


def _word_class(w: bytes) -> str:
    if w == b"\x00" * 8:
        return "zero"
    if 0 not in w:
        return "full"
    return "mixed"


def pack(data: bytes) -> bytes:
    """message.zig:200-271: greedy 256-capped zero runs / no-zero-byte literal runs."""
    if len(data) % 8:
        raise InvalidMessageSize()
    words = [data[i:i + 8] for i in range(0, len(data), 8)]
    out = bytearray()
    i = 0
    n = len(words)
    while i < n:
        cls = _word_class(words[i])
        if cls in ("zero", "full"):
            j = i + 1
            while j < n and j - i < 256 and _word_class(words[j]) == cls:
                j += 1
            run = j - i
            if cls == "zero":
                out += bytes([0x00, run - 1])
            else:
                out += b"\xff" + words[i] + bytes([run - 1]) + b"".join(words[i + 1:j])
            i = j
        else:
            tag = sum(1 << k for k in range(8) if words[i][k])
            out.append(tag)
            out += bytes(b for b in words[i] if b)
            i += 1
    return bytes(out)


def decoded_size(p: bytes) -> int:
    """message.zig:152-191."""
    i, total, n = 0, 0, len(p)
    while i < n:
        t = p[i]
        i += 1
        if t == 0x00:
            if i + 1 > n:
                raise UnexpectedEof()
            total += 8 * (1 + p[i])
            i += 1
        elif t == 0xFF:
            if i + 9 > n:
                raise UnexpectedEof()
            c = p[i + 8]
            i += 9
            if i + 8 * c > n:
                raise UnexpectedEof()
            total += 8 * (1 + c)
            i += 8 * c
        else:
            k = bin(t).count("1")
            if i + k > n:
                raise UnexpectedEof()
            total += 8
            i += k
    return total


def unpack(p: bytes) -> bytes:
    """message.zig:88-145 (size pass first, so errors precede any output)."""
    decoded_size(p)
    out = bytearray()
    i = 0
    while i < len(p):
        t = p[i]
        i += 1
        if t == 0x00:
            out += bytes(8 * (1 + p[i]))
            i += 1
        elif t == 0xFF:
            out += p[i:i + 8]
            c = p[i + 8]
            i += 9
            out += p[i:i + 8 * c]
            i += 8 * c
        else:
            w = bytearray(8)
            for k in range(8):
                if t >> k & 1:
                    w[k] = p[i]
                    i += 1
            out += w
    return bytes(out)


def frame(segments) -> bytes:
    """message.zig:2123-2170 toBytes: segment table + concatenated segments."""
    import struct
    n = len(segments)
    hdr = struct.pack("<I", n - 1) + b"".join(struct.pack("<I", len(s) // 8) for s in segments)
    if n % 2 == 0:
        hdr += b"\x00" * 4
    return hdr + b"".join(segments)


def to_packed_bytes(segments) -> bytes:
    """message.zig:2175-2179 toPackedBytes = packPacked(toBytes())."""
    return pack(frame(segments))


def bench_message_segments(payload_size: int = 4096, list_len: int = 2048):
    """The message bench/packed_unpacked.zig:128-166 (buildMessage, default config,
    payload[i] = 'a' + i % 26 at :302-307) builds, as MessageBuilder segments: one
    segment holding the root pointer, the root struct (2 data words, 2 pointers),
    the text (payload + NUL, word-padded) and the u64 list, allocated in that order.
    Standard capnp pointer encoding (struct pointer: offset << 2 | 0, data words,
    pointer words; list pointer: offset << 2 | 1, element size code | count << 3)."""
    import struct
    payload = bytes(ord("a") + (i % 26) for i in range(payload_size))
    text = payload + b"\x00"
    text_words = (len(text) + 7) // 8
    words = []
    words.append(struct.pack("<IHH", 0 << 2 | 0, 2, 2))                   # root -> struct at word 1
    words.append(struct.pack("<Q", 0x0123456789ABCDEF))                   # data word 0
    words.append(struct.pack("<II", payload_size, 0))                     # data word 1: u32 len at byte 8
    text_at, list_at = 5, 5 + text_words
    words.append(struct.pack("<II", (text_at - 4) << 2 | 1, 2 | (len(text) << 3)))    # ptr 0 (word 3): bytes
    words.append(struct.pack("<II", (list_at - 5) << 2 | 1, 5 | (list_len << 3)))     # ptr 1 (word 4): u64
    seg = b"".join(words) + text + b"\x00" * (8 * text_words - len(text))
    seg += b"".join(struct.pack("<Q", 0 if i % 4 == 0 else (i + 0x0102030405060708) & (2**64 - 1))
                    for i in range(list_len))
    return [seg]


# ---------------------------------------------------------------------------
# Message.validate (message.zig:699-969), restated from the Zig source
# ---------------------------------------------------------------------------

class ValidateError(Exception):
    """Carries the reference's error name (args[0])."""


def _off_words(w):  # decodeOffsetWords, message.zig:11-18
    raw = (w >> 2) & 0x3FFFFFFF
    return raw - (1 << 30) if raw & 0x20000000 else raw


def message_segments(data: bytes):
    """Message.init (message.zig:341-394): list of segment byte strings."""
    import struct
    if len(data) < 4:
        raise ValidateError("EndOfStream")
    n = struct.unpack_from("<I", data, 0)[0]
    if n == 0xFFFFFFFF:
        raise ValidateError("InvalidSegmentCount")
    n += 1
    if n > 512:
        raise ValidateError("SegmentCountLimitExceeded")
    off = 4 * (1 + n + (0 if n % 2 else 1))
    if off > len(data):
        raise ValidateError("TruncatedMessage")
    segs = []
    for i in range(n):
        sz = 8 * struct.unpack_from("<I", data, 4 + 4 * i)[0]
        if off + sz > len(data):
            raise ValidateError("TruncatedMessage")
        segs.append(data[off:off + sz])
        off += sz
    return segs


class _Validator:
    def __init__(self, segs, remaining):
        self.segs = segs
        self.remaining = remaining

    def word(self, seg, pos):
        return int.from_bytes(self.segs[seg][pos:pos + 8], "little")

    def read_word(self, seg, pos):  # :420-425
        if seg >= len(self.segs):
            raise ValidateError("InvalidSegmentId")
        self.bounds(seg, pos, 8)
        return self.word(seg, pos)

    def bounds(self, seg, off, size):  # bounds.zig:10-13
        if off + size > len(self.segs[seg]):
            raise ValidateError("OutOfBounds")

    def consume(self, n):  # :710-713
        if n > self.remaining:
            raise ValidateError("TraversalLimitExceeded")
        self.remaining -= n

    def elements(self, seg, eo, count, dw, pw, nesting):
        if pw == 0 or count == 0:
            return
        for e in range(count):
            ps = eo + e * (dw + pw) * 8 + dw * 8
            for p in range(pw):
                self.pointer(seg, ps + 8 * p, self.word(seg, ps + 8 * p), nesting)

    def pointer(self, seg, pos, w, nesting):  # :715-734
        if w == 0:
            return
        if nesting == 0:
            raise ValidateError("NestingLimitExceeded")
        if seg >= len(self.segs):
            raise ValidateError("InvalidSegmentId")
        t = w & 3
        if t == 0:
            self.struct(seg, pos, w, None, nesting - 1)
        elif t == 1:
            self.list(seg, pos, w, None, nesting - 1)
        elif t == 2:
            self.far(w, nesting - 1)
        else:
            raise ValidateError("InvalidPointer")

    def far(self, w, nesting):  # :736-772 (+ resolveFarLandingPad :430-437)
        double = (w >> 2) & 1
        pad_words = (w >> 3) & 0x1FFFFFFF
        seg = w >> 32
        if seg >= len(self.segs):
            raise ValidateError("InvalidSegmentId")
        landing = pad_words * 8
        self.bounds(seg, landing, 16 if double else 8)
        if not double:
            self.pointer(seg, landing, self.read_word(seg, landing), nesting)
            return
        lw = self.read_word(seg, landing)
        tw = self.read_word(seg, landing + 8)
        if lw & 3 != 2 or (lw >> 2) & 1:
            raise ValidateError("InvalidFarPointer")
        lseg = lw >> 32
        if lseg >= len(self.segs):
            raise ValidateError("InvalidSegmentId")
        eo = ((lw >> 3) & 0x1FFFFFFF) * 8
        if tw & 3 == 0:
            self.ic_tag(lseg, eo, tw, nesting)
        elif tw & 3 == 1:
            self.list(lseg, 0, tw, eo, nesting)
        else:
            raise ValidateError("InvalidFarPointer")

    def struct(self, seg, pos, w, override, nesting):  # :774-812
        dw, pc = (w >> 32) & 0xFFFF, w >> 48
        so = override if override is not None else pos + 8 + _off_words(w) * 8
        if so < 0:
            raise ValidateError("OutOfBounds")
        n = len(self.segs[seg])
        if so > n or (dw + pc) * 8 > n - so:
            raise ValidateError("OutOfBounds")
        self.consume(dw + pc)
        for i in range(pc):
            pp = so + dw * 8 + i * 8
            self.pointer(seg, pp, self.word(seg, pp), nesting)

    def _tag(self, tag, word_count):
        if tag & 3 != 0:
            raise ValidateError("InvalidInlineCompositePointer")
        count = _off_words(tag)
        if count < 0:
            raise ValidateError("InvalidInlineCompositePointer")
        dw, pw = (tag >> 32) & 0xFFFF, tag >> 48
        if word_count is not None and count * (dw + pw) > word_count:
            raise ValidateError("InvalidInlineCompositePointer")
        return count, dw, pw

    def list(self, seg, pos, w, override, nesting):  # :814-897
        es = (w >> 32) & 7
        wc = w >> 35
        if es == 7:
            if override is None:  # validateInlineCompositeList :899-927 via :563-609
                tp = pos + 8 + _off_words(w) * 8
                if tp < 0:
                    raise ValidateError("OutOfBounds")
            else:  # layout B :827-869
                tp = override
            count, dw, pw = self._tag(self.read_word(seg, tp), wc)
            self.bounds(seg, tp + 8, wc * 8)
            self.consume(wc)
            self.elements(seg, tp + 8, count, dw, pw, nesting)
            return
        co = override if override is not None else pos + 8 + _off_words(w) * 8
        if co < 0:
            raise ValidateError("OutOfBounds")
        nbytes = [0, (wc + 7) // 8, wc, 2 * wc, 4 * wc, 8 * wc, 8 * wc][es]
        n = len(self.segs[seg])
        if co > n or nbytes > n - co:
            raise ValidateError("OutOfBounds")
        self.consume((nbytes + 7) // 8)
        if es == 6:
            for i in range(wc):
                self.pointer(seg, co + 8 * i, self.word(seg, co + 8 * i), nesting)

    def ic_tag(self, seg, eo, tag, nesting):  # :929-968
        count, dw, pw = self._tag(tag, None)
        n = len(self.segs[seg])
        if eo > n or count * (dw + pw) * 8 > n - eo:
            raise ValidateError("OutOfBounds")
        self.consume(count * (dw + pw))
        self.elements(seg, eo, count, dw, pw, nesting)


def validate(data: bytes, segment_count_limit=512, traversal_limit_words=8 * 1024 * 1024, nesting_limit=64):
    """Message.init + Message.validate (message.zig:699-708). Returns the traversal
    words consumed; raises ValidateError(name) with the reference's error name."""
    import sys
    segs = message_segments(data)
    if not segs:
        raise ValidateError("EmptyMessage")
    if len(segs) > segment_count_limit:
        raise ValidateError("SegmentCountLimitExceeded")
    if len(segs[0]) < 8:
        raise ValidateError("TruncatedMessage")
    v = _Validator(segs, traversal_limit_words)
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 4 * nesting_limit + 100))
    try:
        v.pointer(0, 0, v.word(0, 0), nesting_limit)
    finally:
        sys.setrecursionlimit(old)
    return traversal_limit_words - v.remaining
