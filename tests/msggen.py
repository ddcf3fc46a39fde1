"""Random Cap'n Proto message trees for the Message.validate tests (test-only).

Builds framed messages (MessageBuilder.toBytes layout, message.zig:2123-2170) whose
pointers use every encoding Message.validate (message.zig:699-969) walks:
  struct pointers                                  makeStructPointer    message.zig:29-35
  list pointers, element sizes 0-6                 makeListPointer      message.zig:37-43
  inline-composite lists (tag word at the target)  resolveInlineCompositeList :563-609
  single far pointers (landing pad = near pointer) validateFarPointer   :749-752
  double far pointers: struct / list tag, layout A (tag in the pad) and layout B
  (list pointer in the pad, tag at the target)     :754-771, :827-869, :929-968
spread over several segments, plus `mutate` which damages random words so that every
error path of the walk is reached.
"""
import struct

import numpy as np

STRUCT, LIST, FAR = 0, 1, 2


def enc_off(off):
    """encodeOffsetWords (message.zig:20-27): 30-bit two's complement."""
    return off & 0x3FFFFFFF


def struct_ptr(off, dw, pw):
    return enc_off(off) << 2 | dw << 32 | pw << 48


def list_ptr(off, es, count):
    return 1 | enc_off(off) << 2 | es << 32 | count << 35


def far_ptr(double, pad_words, seg):
    return 2 | (4 if double else 0) | pad_words << 3 | seg << 32


class Builder:
    def __init__(self, n_segments=1):
        self.segs = [[] for _ in range(n_segments)]

    def alloc(self, seg, n):
        w = self.segs[seg]
        at = len(w)
        w.extend([0] * n)
        return at

    def set(self, seg, pos, word):
        self.segs[seg][pos] = word & 0xFFFFFFFFFFFFFFFF

    def framed(self) -> bytes:
        n = len(self.segs)
        hdr = struct.pack("<I", n - 1) + b"".join(struct.pack("<I", len(s)) for s in self.segs)
        if n % 2 == 0:
            hdr += b"\0" * 4
        body = b"".join(struct.pack(f"<{len(s)}Q", *s) for s in self.segs)
        return hdr + body


class RandomTree:
    """A random object graph written into a Builder, root pointer at segment 0 word 0."""

    def __init__(self, rng, n_segments=None, max_depth=6, max_count=6, far_rate=0.3, null_rate=0.15):
        self.rng = rng
        self.b = Builder(n_segments or int(rng.integers(1, 5)))
        self.max_depth = max_depth
        self.max_count = max_count
        self.far_rate = far_rate
        self.null_rate = null_rate
        self.reads = 1  # words Message.validate reads: pointer slots, landing pads, tags
        self.live = True  # is the pointer being built reached by the walk?
        self.b.alloc(0, 1)
        self.value(0, 0, 0)

    def _seg(self, near_seg):
        n = len(self.b.segs)
        if n > 1 and self.rng.random() < self.far_rate:
            return int(self.rng.integers(0, n))
        return near_seg

    def _data(self, seg, at, n):
        for i in range(n):
            v = int(self.rng.integers(0, 1 << 63)) if self.rng.random() < 0.7 else 0
            self.b.set(seg, at + i, v)

    def value(self, seg, pos, depth):
        """Write a random pointer at (seg, pos) and build what it points to."""
        rng = self.rng
        if depth >= self.max_depth or rng.random() < self.null_rate:
            return  # null pointer
        kind = rng.choice(["struct", "list", "ptrlist", "composite"], p=[0.35, 0.3, 0.15, 0.2])
        t = self._seg(seg)
        mc = self.max_count
        if kind == "struct":
            dw, pw = int(rng.integers(0, 4)), int(rng.integers(0, 4))
            content = self.b.alloc(t, dw + pw)
            self._data(t, content, dw)
            live = self.live
            self.live = self.link(seg, pos, t, content, lambda off: struct_ptr(off, dw, pw), ("struct", dw, pw)) \
                and live
            self.reads += pw if self.live else 0
            for i in range(pw):
                self.value(t, content + dw + i, depth + 1)
            self.live = live
        elif kind == "list":
            es = int(rng.integers(0, 6))
            count = int(rng.integers(0, 4 * mc))
            nbytes = [0, (count + 7) // 8, count, 2 * count, 4 * count, 8 * count][es]
            words = (nbytes + 7) // 8
            content = self.b.alloc(t, words)
            self._data(t, content, words)
            self.link(seg, pos, t, content, lambda off: list_ptr(off, es, count), ("list", es, count))
        elif kind == "ptrlist":
            count = int(rng.integers(0, mc))
            content = self.b.alloc(t, count)
            self.link(seg, pos, t, content, lambda off: list_ptr(off, 6, count), ("list", 6, count))
            self.reads += count if self.live else 0
            for i in range(count):
                self.value(t, content + i, depth + 1)
        else:
            count = int(rng.integers(0, mc))
            dw, pw = int(rng.integers(0, 3)), int(rng.integers(0, 3))
            wc = count * (dw + pw)
            layout_a = t != seg and rng.random() < 0.5  # tag in the double-far pad
            if layout_a:
                content = self.b.alloc(t, wc)
                tag = struct_ptr(count, dw, pw)
                pad_seg = int(rng.integers(0, len(self.b.segs)))
                pad = self.b.alloc(pad_seg, 2)
                self.b.set(pad_seg, pad, far_ptr(False, content, t))
                self.b.set(pad_seg, pad + 1, tag)
                self.b.set(seg, pos, far_ptr(True, pad, pad_seg))
                self.reads += 2 if self.live else 0
            else:
                self.reads += 1 if self.live else 0
                tag_at = self.b.alloc(t, 1 + wc)
                self.b.set(t, tag_at, struct_ptr(count, dw, pw))
                content = tag_at + 1
                self.link(seg, pos, t, tag_at, lambda off: list_ptr(off, 7, wc), ("list", 7, wc))
            self.reads += count * pw if self.live else 0
            for e in range(count):
                base = content + e * (dw + pw)
                self._data(t, base, dw)
                for i in range(pw):
                    self.value(t, base + dw + i, depth + 1)

    def link(self, seg, pos, t, content, near, far_tag):
        """Point (seg, pos) at `content` in segment t: near pointer, single far (landing
        pad = near pointer before the content) or double far (pad = far + tag). Returns
        whether Message.validate goes on into the content's pointers."""
        if t == seg:
            self.b.set(seg, pos, near(content - pos - 1))
            return True
        if self.rng.random() < 0.5:
            pad = self.b.alloc(t, 1)
            self.b.set(t, pad, near(content - pad - 1))
            self.b.set(seg, pos, far_ptr(False, pad, t))
            self.reads += 1 if self.live else 0
            return True
        self.reads += 2 if self.live else 0
        pad_seg = int(self.rng.integers(0, len(self.b.segs)))
        pad = self.b.alloc(pad_seg, 2)
        self.b.set(pad_seg, pad, far_ptr(False, content, t))
        kind, a, c = far_tag
        self.b.set(pad_seg, pad + 1, struct_ptr(0, a, c) if kind == "struct" else list_ptr(0, a, c))
        self.b.set(seg, pos, far_ptr(True, pad, pad_seg))
        # a struct tag behind a double far is read as an inline-composite tag of count 0
        # (its offset field, validateFarPointer :765-767): the walk stops there
        return kind != "struct"

    def framed(self) -> bytes:
        return self.b.framed()


def random_message(rng, **kw) -> bytes:
    return RandomTree(rng, **kw).framed()


def header_bytes(msg: bytes) -> int:
    n = struct.unpack_from("<I", msg, 0)[0] + 1
    return 4 * (1 + n + (0 if n % 2 else 1))


def mutate(rng, msg: bytes, n_edits=None) -> bytes:
    """Damage a framed message: overwrite random bits, bytes, fields of pointer words
    or whole words after the segment table (and, rarely, the table itself)."""
    b = bytearray(msg)
    hdr = header_bytes(msg) if len(msg) >= 4 else 0
    n_edits = n_edits or int(rng.integers(1, 4))
    for _ in range(n_edits):
        if len(b) <= hdr or rng.random() < 0.03:
            if len(b) >= 4:
                i = int(rng.integers(0, min(len(b), max(hdr, 4))))
                b[i] ^= 1 << int(rng.integers(0, 8))
            continue
        w = hdr + 8 * int(rng.integers(0, (len(b) - hdr) // 8)) if len(b) - hdr >= 8 else hdr
        r = rng.random()
        if w + 8 > len(b):
            continue
        word = int.from_bytes(b[w:w + 8], "little")
        if r < 0.35:
            word ^= 1 << int(rng.integers(0, 64))
        elif r < 0.5:
            word ^= 3  # pointer type
        elif r < 0.65:
            word ^= int(rng.integers(1, 1 << 30)) << 2  # offset / landing pad
        elif r < 0.8:
            word ^= int(rng.integers(1, 1 << 16)) << int(rng.choice([32, 35, 48]))  # sizes / counts / seg id
        else:
            word = int(rng.integers(0, 1 << 63)) * 2 + int(rng.integers(0, 2))
        b[w:w + 8] = (word & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")
    return bytes(b)


def corpus(seed, n, mutate_rate=0.7, **kw):
    """n framed messages: random trees, most of them damaged."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        m = random_message(rng, **kw)
        if rng.random() < mutate_rate:
            m = mutate(rng, m)
        out.append(m)
    return out


def deep_chain(depth: int) -> bytes:
    """A chain of `depth` structs (0 data words, 1 pointer), the last one (1, 0)."""
    b = Builder(1)
    b.alloc(0, 1)
    pos = 0
    for d in range(depth):
        last = d == depth - 1
        at = b.alloc(0, 1)
        b.set(0, pos, struct_ptr(at - pos - 1, 1 if last else 0, 0 if last else 1))
        pos = at
    return b.framed()


def deep_mixed(rng, depth: int, n_segments: int = 3) -> bytes:
    """A spine of `depth` pointer levels of mixed kinds: structs (extra null pointers and
    data words beside the one that goes on), pointer lists and inline-composite lists (the
    spine through one element), each link near or through a single far pointer (which
    spends one more nesting level, validateFarPointer :736-752). The spine ends in a struct
    with one data word."""
    b = Builder(n_segments)
    b.alloc(0, 1)
    seg, pos = 0, 0
    for d in range(depth):
        last = d == depth - 1
        t = seg if rng.random() < 0.6 else int(rng.integers(0, n_segments))
        kind = "end" if last else str(rng.choice(["struct", "ptrlist", "composite"]))
        if kind in ("end", "struct"):
            dw = 1 if last else int(rng.integers(0, 2))
            pw = 0 if last else int(rng.integers(1, 3))
            content = b.alloc(t, dw + pw)
            for i in range(dw):
                b.set(t, content + i, int(rng.integers(0, 1 << 63)))
            near = lambda off, dw=dw, pw=pw: struct_ptr(off, dw, pw)
            nxt = content + dw + (int(rng.integers(0, pw)) if pw else 0)
        elif kind == "ptrlist":
            count = int(rng.integers(1, 3))
            content = b.alloc(t, count)
            near = lambda off, count=count: list_ptr(off, 6, count)
            nxt = content + int(rng.integers(0, count))
        else:
            count, dw = int(rng.integers(1, 3)), int(rng.integers(0, 2))
            wc = count * (dw + 1)
            tag_at = b.alloc(t, 1 + wc)
            b.set(t, tag_at, struct_ptr(count, dw, 1))
            content = tag_at
            near = lambda off, wc=wc: list_ptr(off, 7, wc)
            nxt = tag_at + 1 + int(rng.integers(0, count)) * (dw + 1) + dw
        if t == seg:
            b.set(seg, pos, near(content - pos - 1))
        else:  # single far: the landing pad is a near pointer in the target segment
            pad = b.alloc(t, 1)
            b.set(t, pad, near(content - pad - 1))
            b.set(seg, pos, far_ptr(False, pad, t))
        seg, pos = t, nxt
    return b.framed()
