#!/usr/bin/env python3
"""Framer dispatch rule (verdict r4 item 5): per read call, the device
framer session (capnp_packed_framer_readv: gather, H2D, walk, decode, D2H of the frames) against
the CPU framer on one host core (oracle_read_stream: readPackedMessage, reader.zig:84-156, over
each connection's buffered bytes until no whole message is left, as Connection.handleRead's loop
does, level2/connection.zig:153-203).

Two shapes, p = 0.5 messages of 4 KiB framed (one segment), or one large message:
  many:  N connections x 16 messages per read call, N = 1 .. 4096 (a batch of connections that
         each received 16 whole messages): bytes per call = N x 16 x ~2.6 KB packed;
  split: one connection, one message of M framed bytes arriving in 64 KiB reads. The device
         session resumes its walk across reads (every byte uploaded and walked once); the CPU
         framer keeps the bytes and retries readPackedMessage from the message start on every
         read, as a Framer over a packed stream does when the message is incomplete.
Both sides get whole host buffers in and out: the device call is the C-ABI entry itself (ctypes,
preallocated page-locked frames buffer), not the Python mirror. Prints one JSON object; the
threshold per shape is the smallest size from which the device call is faster.
Usage: python3 scripts/framer_crossover.py [--reps 7]
"""
import argparse
import ctypes
import json
import os
import statistics
import struct
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "capnp-zig_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402
import oracle  # noqa: E402

def packed_messages(n, framed, seed, thr=128):
    """n one-segment messages of `framed` bytes (header + words), packed, on the host."""
    words = framed // 8 - 1
    dev = torch.device("cuda", 0)
    d_fr = cp.generate(n, framed, seed=seed, zero_thresh=thr, device=dev)
    d_fr.view(n, framed)[:, :8] = torch.tensor(list(struct.pack("<II", 0, words)), dtype=torch.uint8, device=dev)
    off, ln = cp.uniform_layout(n, framed, device=dev)
    slot = cp.encode_bound(framed)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    d_pk = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.zeros(n, dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    cp.encode_batch(d_fr, off, ln, d_pk, pk_off, pk_cap, plen, pst)
    torch.cuda.synchronize()
    pk, pl = d_pk.cpu().numpy(), plen.cpu().numpy()
    return [pk[i * slot:i * slot + int(pl[i])].tobytes() for i in range(n)]


class Device:
    """One framer session with its page-locked frames buffer, called through the C-ABI."""

    def __init__(self, n_conns, total):
        L = cp.lib()
        self.L, self.n = L, n_conns
        h = ctypes.c_void_p()
        st = L.capnp_packed_framer_create(n_conns, ctypes.byref(h))
        assert st == 0, st
        self.h = h
        self.cap = 2 * total + (1 << 16)
        self.frames = torch.empty(self.cap, dtype=torch.uint8, pin_memory=True)
        self.max_frames = max(1024, total // 2 + 64)
        self.f_off = np.zeros(self.max_frames, dtype=np.uint64)
        self.f_len = np.zeros(self.max_frames, dtype=np.uint64)
        self.f_conn = np.zeros(self.max_frames, dtype=np.uint32)
        self.status = np.zeros(n_conns, dtype=np.int32)
        self.ptrs = (ctypes.c_char_p * n_conns)()
        self.lens = np.zeros(n_conns, dtype=np.uint64)

    def readv(self, reads):
        """reads: list of bytes per connection (b"" = none); returns the frames popped."""
        for c, d in enumerate(reads):
            self.ptrs[c] = d if d else None
            self.lens[c] = len(d)
        nf = ctypes.c_uint32(0)
        st = self.L.capnp_packed_framer_readv(
            self.h, self.ptrs, self.lens.ctypes.data, self.frames.data_ptr(), self.cap, self.f_off.ctypes.data,
            self.f_len.ctypes.data, self.f_conn.ctypes.data, self.max_frames, self.status.ctypes.data,
            ctypes.byref(nf))
        assert st == 0, st
        return nf.value

    def close(self):
        self.L.capnp_packed_framer_destroy(self.h)


def olib():
    O = oracle.lib()
    O.oracle_read_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    O.oracle_read_stream.restype = ctypes.c_size_t
    return O


def addr(b):
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if isinstance(b, bytes) else \
        ctypes.addressof((ctypes.c_char * len(b)).from_buffer(b))


def cpu_read(bufs, out):
    """oracle_read_stream over each connection's bytes; returns the frames read."""
    O = olib()
    used, tot = ctypes.c_size_t(), ctypes.c_size_t()
    frames = 0
    for b in bufs:
        if b:
            frames += O.oracle_read_stream(addr(b), len(b), out.ctypes.data, out.size, ctypes.byref(used),
                                           ctypes.byref(tot))
    return frames


def many(reps):
    msgs = 16
    pool = packed_messages(4096 * msgs, 4096, seed=0xC0DE0009)
    out = np.zeros(64 << 20, dtype=np.uint8)
    rows = []
    n = 1
    while n <= 4096:
        bufs = [b"".join(pool[c * msgs:(c + 1) * msgs]) for c in range(n)]
        total = sum(len(b) for b in bufs)
        dev = Device(n, total)
        dev.readv(bufs)  # first read: the session's allocations
        g = []
        for _ in range(reps):
            t = time.perf_counter()
            nf = dev.readv(bufs)
            g.append(time.perf_counter() - t)
            assert nf == n * msgs, (nf, n * msgs)
        dev.close()
        c = []
        for _ in range(reps):
            t = time.perf_counter()
            fr = cpu_read(bufs, out)
            c.append(time.perf_counter() - t)
            assert fr == n * msgs
        rows.append({"connections": n, "messages": n * msgs, "packed_bytes": total,
                     "device_us": round(statistics.median(g) * 1e6, 1),
                     "cpu_1core_us": round(statistics.median(c) * 1e6, 1)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
        n *= 2
    return rows


def split(reps, read_bytes=65536):
    rows = []
    out = np.zeros(80 << 20, dtype=np.uint8)
    O = olib()
    for framed in (1 << 16, 1 << 18, 1 << 20, 1 << 22, 1 << 24):
        stream = packed_messages(1, framed, seed=0xC0DE000A)[0]
        reads = [stream[i:i + read_bytes] for i in range(0, len(stream), read_bytes)]
        g = []
        dev = Device(1, len(stream))  # one long-lived session; rep 0 pays its allocations
        for r in range(reps + 1):
            t = time.perf_counter()
            nf = sum(dev.readv([piece]) for piece in reads)
            dt = time.perf_counter() - t
            assert nf == 1
            if r:
                g.append(dt)
        dev.close()
        c = []
        for r in range(max(1, reps // 2) if framed <= (1 << 20) else 1):
            buf = bytearray()
            t = time.perf_counter()
            frames = 0
            for piece in reads:  # the Framer keeps the bytes; readPackedMessage from the start
                buf += piece
                used, tot = ctypes.c_size_t(), ctypes.c_size_t()
                frames += O.oracle_read_stream(addr(buf), len(buf), out.ctypes.data, out.size, ctypes.byref(used),
                                               ctypes.byref(tot))
            c.append(time.perf_counter() - t)
            assert frames == 1
        rows.append({"framed_bytes": framed, "packed_bytes": len(stream), "reads": len(reads),
                     "device_us": round(statistics.median(g) * 1e6, 1),
                     "cpu_1core_us": round(statistics.median(c) * 1e6, 1)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    return rows


def threshold(rows, key):
    for i, r in enumerate(rows):
        if all(x["device_us"] < x["cpu_1core_us"] for x in rows[i:]):
            return r[key]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    m = many(a.reps)
    s = split(a.reps)
    print(json.dumps({"many": m, "split": s,
                      "threshold_many_packed_bytes": threshold(m, "packed_bytes"),
                      "threshold_split_framed_bytes": threshold(s, "framed_bytes"),
                      "note": "device: capnp_packed_framer_readv per read call (C-ABI, page-locked frames); "
                              "cpu: oracle_read_stream on one core (readPackedMessage loop per connection)"}))


if __name__ == "__main__":
    main()
