#!/usr/bin/env python3
"""Dev-only host model of decode_stream_kernel's per-lane logic (packed_kernels.hip, DESIGN.md
§2.3b): the 80-B ring per round (block k-1's last piece + block k, stale past the last block),
the walk steps with their u16 entries (tag << 8 | ring offset of the word's bytes), zero-run
jobs, words past the capacity counted only, and the store phase's expansion from the ring.
Checked against the oracle (tests/oracle.py, message.zig:88-191) on random and adversarial
units. Usage: python3 scripts/dev/sim_stream.py [n_units]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import oracle  # noqa: E402

K, ZJOB, DEAD = 16, 16, 0xFFFFFFF0
EOF_, SPACE, OK = 2, 4, 0


def expand(ring, e):
    tg, dd = e >> 8, e & 0xFF
    data = bytes(ring[dd:dd + 8])
    if tg == 0xFF:
        return data
    out, j = bytearray(8), 0
    for b in range(8):
        if (tg >> b) & 1:
            out[b] = data[j]
            j += 1
    return bytes(out)


def decode(packed: bytes, cap: int, s: int = 0):
    P = len(packed)
    mem = bytes(s) + packed + bytes(96)       # aligned space: unit byte i at s + i
    end = s + P
    maxr = (end + 63) >> 6 if P else 0
    capw = cap >> 3
    out = bytearray(cap)
    pos, lit_end, zrem, wc, st = (s if P else DEAD), 0, 0, 0, OK
    ring = bytearray(80)
    for k in range(maxr + 1):
        if k > 0:
            ring[0:16] = ring[64:80]
        if k < maxr:
            ring[16:80] = mem[64 * k:64 * k + 64]
        ob = 64 * k
        lim = min(ob + 48, end)
        while True:
            w0, ents, zjob = wc, [], 0
            for i in range(K):
                inz = zrem != 0
                act = zjob == 0 and (inz or pos < lim)
                if not act:
                    break
                o = (pos + 16 - ob) & 63
                t, b1, c9 = ring[o], ring[o + 1], ring[o + 9]
                lit = (not inz) and pos < lit_end
                rec = not inz and not lit
                z, f = t == 0, t == 0xFF
                ln = 8 if lit else 1 + bin(t).count("1") + (1 if (z or f) else 0)
                lend = pos + 10 + 8 * c9
                eof = rec and (pos + ln > end or (f and lend > end))
                tg = 0 if inz else (0xFF if lit else t)
                dd = o if lit else o + 1
                em = not eof
                wn = wc + (1 if em else 0)
                zr = rec and not eof and z and b1 != 0
                bulk = zr and wn >= capw
                job = zr and not bulk and b1 >= ZJOB
                zrem = zrem - 1 if inz else (b1 if (zr and not bulk and not job) else 0)
                zjob = b1 if job else 0
                wc = wn + (b1 if bulk else 0)
                if rec and f:
                    lit_end = lend
                pos = DEAD if eof else (pos if inz else pos + ln)
                if eof:
                    st = EOF_
                if em:
                    ents.append((tg << 8) | dd)
            lu = min(len(ents), capw - w0) if w0 < capw else 0
            for i in range(lu):
                out[8 * (w0 + i):8 * (w0 + i) + 8] = expand(ring, ents[i])
            if zjob:
                hi = min(wc + zjob, capw)
                out[8 * wc:8 * hi] = bytes(8 * (hi - wc))
            wc += zjob
            if not (zrem != 0 or pos < lim):
                break
    if st != OK:
        return st, 0, out
    return (SPACE if wc > capw else OK), 8 * wc, out


def check(packed, cap, s):
    st, ln, out = decode(packed, cap, s)
    ost, ref = oracle.unpack(packed)
    want = ost if ost != oracle.OK or len(ref) <= cap else oracle.OUT_OF_SPACE
    assert st == want, (st, want, len(packed), cap, s)
    if want == OK:
        assert ln == len(ref) and bytes(out[:ln]) == ref, (len(packed), cap, s)
    elif want == SPACE:
        assert ln == len(ref)
        assert bytes(out[:cap - cap % 8]) == ref[:cap - cap % 8]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    rng = np.random.default_rng(1)
    for i in range(n):
        kind = i % 6
        words = int(rng.integers(0, 700))
        if kind == 5:  # raw random bytes: truncations, odd records
            p = rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
        else:
            thr = [0.02, 0.1, 0.5, 0.9, 0.99][kind]
            b = rng.integers(1, 256, 8 * words, dtype=np.uint8)
            b[rng.random(8 * words) < thr] = 0
            if kind == 4 and words:
                b[: 8 * int(rng.integers(0, words))] = 0  # long zero runs (jobs)
            st, p = oracle.pack(b.tobytes())
            if i % 7 == 3 and p:
                p = p[:-int(rng.integers(1, min(len(p), 12) + 1))]
        ost, ref = oracle.unpack(p)
        cap = len(ref) if ost == 0 else 8 * 4096
        if i % 5 == 2 and ost == 0 and len(ref) >= 8:
            cap = len(ref) - 8 * int(rng.integers(1, len(ref) // 8 + 1))
        check(p, cap, int(rng.integers(0, 16)))
    print(f"sim ok: {n} units")


if __name__ == "__main__":
    main()
