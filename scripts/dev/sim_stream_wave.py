#!/usr/bin/env python3
"""Dev-only: decode_stream_kernel modelled a wave at a time (64 lanes in lockstep, idle lanes
executing the step with act = false, as on the device), on the adversarial/fuzz corpus of
tests/test_gpu_parity.py::test_batch_decode_adversarial_and_fuzz. The per-lane model
(sim_stream.py) cannot see state that idle lanes change; this one found the round-4 hang
(idle lanes advancing pos past kDsDead and wrapping). Usage: sim_stream_wave.py [--unguarded]"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import oracle  # noqa: E402
from sim_stream import expand, K, ZJOB, DEAD, EOF_, SPACE, OK  # noqa: E402

M32 = 0xFFFFFFFF
GUARD = "--unguarded" not in sys.argv  # the pre-fix step (hangs)

def decode_wave(units):  # units: list of (packed, cap, s), <= 64
    L = len(units)
    mems, ends, capw, outs = [], [], [], []
    for p, cap, s in units:
        mems.append(bytes(s) + p + bytes(random.getrandbits(8) for _ in range(200))); ends.append(s + len(p) if p else 0)
        capw.append(cap >> 3); outs.append(bytearray(cap))
    maxr = max((e + 63) >> 6 for e in ends)
    pos = [units[l][2] if units[l][0] else DEAD for l in range(L)]
    lit_end = [0]*L; zrem=[0]*L; wc=[0]*L; st=[OK]*L
    rings = [bytearray(80) for _ in range(L)]
    subrounds = 0
    for k in range(maxr + 1):
        for l in range(L):
            if k > 0: rings[l][0:16] = rings[l][64:80]
            if k < maxr:
                npc = (ends[l] + 15) >> 4
                for q in range(4):
                    pc = min(4*k+q, max(npc-1, 0))
                    rings[l][16+16*q:32+16*q] = mems[l][16*pc:16*pc+16] if npc else bytes(16)
        ob = 64 * k
        lim = [min(ob + 48, ends[l]) for l in range(L)]
        while True:
            subrounds += 1
            if subrounds > 100000: raise RuntimeError("hang")
            w0 = wc[:]; nent=[0]*L; zjob=[0]*L; ents=[[None]*K for _ in range(L)]
            for i in range(K):
                acts = [zjob[l]==0 and (zrem[l]!=0 or pos[l] < lim[l]) for l in range(L)]
                if not any(acts): break
                for l in range(L):
                    ring = rings[l]; act = acts[l]; inz = zrem[l] != 0
                    o = (pos[l] + 16 - ob) & 63
                    t, b1, c9 = ring[o], ring[o+1], ring[o+9]
                    lit = (not inz) and pos[l] < lit_end[l]
                    rec = act and not inz and not lit
                    z, f = t == 0, t == 0xFF
                    ln = 8 if lit else 1 + bin(t).count("1") + (1 if (z or f) else 0)
                    lend = (pos[l] + 10 + 8*c9) & M32
                    eof = rec and (((pos[l]+ln)&M32) > ends[l] or (f and lend > ends[l]))
                    tg = 0 if inz else (0xFF if lit else t)
                    dd = o if lit else o + 1
                    ents[l][i] = (tg << 8) | dd
                    em = act and not eof
                    wn = wc[l] + (1 if em else 0)
                    zr = rec and not eof and z and b1 != 0
                    bulk = zr and wn >= capw[l]
                    job = zr and not bulk and b1 >= ZJOB
                    zrem[l] = zrem[l]-1 if inz else (b1 if (zr and not bulk and not job) else 0)
                    if GUARD: zjob[l] = b1 if job else zjob[l]
                    else: zjob[l] = b1 if job else 0
                    wc[l] = wn + (b1 if bulk else 0)
                    if rec and f: lit_end[l] = lend
                    if GUARD: pos[l] = DEAD if eof else (pos[l] if (inz or not act) else (pos[l]+ln)&M32)
                    else: pos[l] = DEAD if eof else (pos[l] if inz else (pos[l]+ln)&M32)
                    if eof: st[l] = EOF_
                    if em: nent[l] = i + 1
            for l in range(L):
                lu = min(nent[l], capw[l]-w0[l]) if w0[l] < capw[l] else 0
                for i in range(lu):
                    outs[l][8*(w0[l]+i):8*(w0[l]+i)+8] = expand(rings[l], ents[l][i])
                if zjob[l]:
                    hi = min(wc[l]+zjob[l], capw[l]); outs[l][8*wc[l]:8*hi] = bytes(8*(hi-wc[l]))
                wc[l] += zjob[l]
            if not any(zrem[l]!=0 or pos[l] < lim[l] for l in range(L)): break
    res = []
    for l in range(L):
        if st[l] != OK: res.append((st[l], 0, outs[l]))
        else: res.append((SPACE if wc[l] > capw[l] else OK, 8*wc[l], outs[l]))
    return res

units = [bytes.fromhex(h) for h in (
    "", "01", "00", "0000", "00ff", "ff", "ff01020304", "ff0102030405060708",
    "ff010203040506070800", "ff010203040506070801", "ff010203040506070801aabb",
    "ff0102030405060708ff", "fe0102", "80", "000001", "00000000", "ffffffffffffffffffff",
    "0003", "0001ff010203040506070800", "03aa", "10010000", "0001")]
rng = random.Random(0xA7C41E59)
units += [bytes(rng.randrange(256) for _ in range(rng.randrange(160))) for _ in range(1024)]
# unaligned placement as device_units (align=1)
offs, p = [], 0
for u in units: offs.append(p); p += len(u)
lanes = []
for u, o in zip(units, offs):
    st, ref = oracle.unpack(u)
    lanes.append((u, len(ref) if st == OK else 0, o & 15))
bad = 0
for w in range(0, len(lanes), 64):
    res = decode_wave(lanes[w:w+64])
    for j, (st, ln, out) in enumerate(res):
        u = lanes[w+j][0]; ost, ref = oracle.unpack(u)
        if ost != st or (st == OK and bytes(out[:ln]) != ref):
            bad += 1
# mixed corpus: encoded units (zero jobs, long literals), truncations, tight capacities
import numpy as np  # noqa: E402
g = np.random.default_rng(3)
mix = []
for i in range(1280):
    kind = i % 6
    words = int(g.integers(0, 120))
    if kind == 5:
        p = g.integers(0, 256, int(g.integers(0, 300)), dtype=np.uint8).tobytes()
    else:
        b = g.integers(1, 256, 8 * words, dtype=np.uint8)
        b[g.random(8 * words) < [0.02, 0.1, 0.5, 0.9, 0.99][kind]] = 0
        if kind == 4 and words:
            b[: 8 * int(g.integers(0, words))] = 0
        p = oracle.pack(b.tobytes())[1]
        if i % 7 == 3 and p:
            p = p[:-int(g.integers(1, min(len(p), 12) + 1))]
    ost, ref = oracle.unpack(p)
    cap = len(ref) if ost == OK else 8 * 64
    if i % 5 == 2 and ost == OK and len(ref) >= 8:
        cap = len(ref) - 8 * int(g.integers(1, len(ref) // 8 + 1))
    mix.append((p, cap, int(g.integers(0, 16))))
for w in range(0, len(mix), 64):
    for j, (st, ln, out) in enumerate(decode_wave(mix[w:w + 64])):
        p, cap = mix[w + j][0], mix[w + j][1]
        ost, ref = oracle.unpack(p)
        want = ost if ost != OK or len(ref) <= cap else SPACE
        if st != want or (st == OK and bytes(out[:ln]) != ref) or \
                (st == SPACE and (ln != len(ref) or bytes(out[:cap - cap % 8]) != ref[:cap - cap % 8])):
            bad += 1
print("bad", bad)
sys.exit(1 if bad else 0)
