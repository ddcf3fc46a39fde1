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
