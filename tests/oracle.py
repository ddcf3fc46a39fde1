"""ctypes loader for the CPU oracle (oracle/liboracle.so). Test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

OK, INVALID_MESSAGE_SIZE, UNEXPECTED_EOF, OVERFLOW, OUT_OF_SPACE, INVALID_ARGUMENT = range(6)

_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_szp = ctypes.POINTER(ctypes.c_size_t)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_pack.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, _szp]
        L.oracle_unpack.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, _szp]
        L.oracle_estimate_unpacked_size.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _szp]
        L.oracle_message_init.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                          _u64p, _u64p, ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_read_packed_message.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                 ctypes.c_size_t, _szp, _szp]
        batch = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_pack_batch.argtypes = batch
        L.oracle_unpack_batch.argtypes = batch
        L.fast_pack_batch.argtypes = batch    # oracle/packed_fast.c (bench.py's cpu_baseline)
        L.fast_unpack_batch.argtypes = batch
        L.oracle_generate.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int]
        L.oracle_mix64.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_mix64.restype = ctypes.c_uint64
        L.oracle_word_has_zero_byte.argtypes = [ctypes.c_uint64]
        L.oracle_validate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint64, _u64p]
        _lib = L
    return _lib


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), max(1, len(b)))


def pack(data: bytes):
    """(status, packed bytes) — message.zig:200-271."""
    src = _buf(data)
    cap = 10 * (len(data) // 8) + 16
    dst = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t()
    st = lib().oracle_pack(src, len(data), dst, cap, ctypes.byref(n))
    return st, (dst.raw[:n.value] if st == OK else b"")


def decoded_size(p: bytes):
    src = _buf(p)
    n = ctypes.c_size_t()
    st = lib().oracle_estimate_unpacked_size(src, len(p), ctypes.byref(n))
    return st, n.value


def unpack(p: bytes):
    """(status, unpacked bytes) — message.zig:88-145."""
    st, size = decoded_size(p)
    if st != OK:
        return st, b""
    src = _buf(p)
    dst = ctypes.create_string_buffer(max(1, size))
    n = ctypes.c_size_t()
    st = lib().oracle_unpack(src, len(p), dst, size, ctypes.byref(n))
    return st, dst.raw[:n.value]


def message_init(data: bytes, max_segs=512):
    """(code, [(off, len), ...]) — message.zig:341-394 segment table parse."""
    src = _buf(data)
    off = (ctypes.c_uint64 * max_segs)()
    ln = (ctypes.c_uint64 * max_segs)()
    cnt = ctypes.c_uint32()
    rc = lib().oracle_message_init(src, len(data), max_segs, off, ln, ctypes.byref(cnt))
    return rc, [(off[i], ln[i]) for i in range(min(cnt.value, max_segs))]


def read_packed_message(p: bytes, cap=1 << 20):
    """(code, framed bytes, consumed) — reader.zig:84-156."""
    src = _buf(p)
    dst = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t()
    used = ctypes.c_size_t()
    rc = lib().oracle_read_packed_message(src, len(p), dst, cap, ctypes.byref(n), ctypes.byref(used))
    return rc, dst.raw[:n.value], used.value


def validate(data: bytes, segment_count_limit=512, traversal_limit_words=8 * 1024 * 1024, nesting_limit=64):
    """(status, traversal words consumed) — message.zig:699-969 Message.validate of a
    framed message (Message.init first); status codes are include/capnp_packed.h's."""
    src = _buf(data)
    words = ctypes.c_uint64()
    st = lib().oracle_validate(src, len(data), segment_count_limit, traversal_limit_words, nesting_limit,
                               ctypes.byref(words))
    return st, words.value


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _batch_bufs(n, out_off):
    """(out, out_len, status) for a batch call; pass them back as bufs= to reuse them (the CPU
    baseline does, so that its timed calls do not fault in fresh pages)."""
    return (np.zeros(int(out_off[-1]) + 16, dtype=np.uint8), np.zeros(n, dtype=np.uint64),
            np.zeros(n, dtype=np.int32))


def pack_batch(inp: np.ndarray, in_off: np.ndarray, out_off: np.ndarray, threads=0, bufs=None):
    n = len(in_off) - 1
    out, out_len, status = bufs if bufs is not None else _batch_bufs(n, out_off)
    lib().oracle_pack_batch(_ptr(inp), _ptr(in_off), n, _ptr(out), _ptr(out_off), _ptr(out_len),
                            _ptr(status), threads)
    return out, out_len, status


def unpack_batch(inp: np.ndarray, in_off: np.ndarray, out_off: np.ndarray, threads=0, bufs=None):
    n = len(in_off) - 1
    out, out_len, status = bufs if bufs is not None else _batch_bufs(n, out_off)
    lib().oracle_unpack_batch(_ptr(inp), _ptr(in_off), n, _ptr(out), _ptr(out_off), _ptr(out_len),
                              _ptr(status), threads)
    return out, out_len, status


def fast_pack_batch(inp: np.ndarray, in_off: np.ndarray, out_off: np.ndarray, threads=0, bufs=None):
    """pack_batch on oracle/packed_fast.c (the CPU baseline's word-at-a-time port)."""
    n = len(in_off) - 1
    out, out_len, status = bufs if bufs is not None else _batch_bufs(n, out_off)
    lib().fast_pack_batch(_ptr(inp), _ptr(in_off), n, _ptr(out), _ptr(out_off), _ptr(out_len), _ptr(status), threads)
    return out, out_len, status


def fast_unpack_batch(inp: np.ndarray, in_off: np.ndarray, out_off: np.ndarray, threads=0, bufs=None):
    """unpack_batch on oracle/packed_fast.c."""
    n = len(in_off) - 1
    out, out_len, status = bufs if bufs is not None else _batch_bufs(n, out_off)
    lib().fast_unpack_batch(_ptr(inp), _ptr(in_off), n, _ptr(out), _ptr(out_off), _ptr(out_len), _ptr(status),
                            threads)
    return out, out_len, status


def generate(n_units, unit_bytes, seed, zero_thresh, unit_base=0, threads=0) -> np.ndarray:
    out = np.empty(n_units * unit_bytes, dtype=np.uint8)
    lib().oracle_generate(_ptr(out), n_units, unit_bytes, unit_base, seed, zero_thresh, threads)
    return out
