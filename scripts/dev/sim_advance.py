#!/usr/bin/env python3
"""Dev model (round 6): lane-steps of the words decoder per unit under two round schedules.
A: block-synchronous rounds (the shipped kernel): round k gives every lane block k; the round
   lasts max over the wave's lanes of the words whose source lies in block k's window, cut in
   sub-rounds of S steps (the round costs the longest lane's steps).
B: per-unit block advance: every sub-round (S steps) is a round boundary; a lane whose next
   source has left its block's window takes its next block there, else keeps its block; a lane
   idles from the step its window is exhausted to the sub-round's end.
Zero-run words need no bytes (they are emitted in any round). Prints words / lane-steps.
Usage: python3 scripts/dev/sim_advance.py [units] [S]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle  # noqa: E402


def word_src(p):
    """per output word: the source position whose bytes it needs (None for zero-run words)"""
    out, i, n = [], 0, len(p)
    while i < n:
        t = p[i]
        if t == 0:
            out.append(i)
            out += [None] * p[i + 1]
            i += 2
        elif t == 0xFF:
            out.append(i)
            c = p[i + 9]
            out += [i + 10 + 8 * j for j in range(c)]
            i += 10 + 8 * c
        else:
            out.append(i)
            i += 1 + bin(t).count("1")
    return out


def lim_of(pos):  # the words decoder's window: block k takes sources below 64k + 52 (from -12)
    return (pos + 12) // 64


def sched_a(units, S):
    steps = 0
    srcs = [word_src(p) for p in units]
    R = max((len(p) + 12) // 64 + 1 for p in units) + 1
    ptr = [0] * len(units)
    for k in range(R):
        cnt = []
        for u, s in enumerate(srcs):
            c = 0
            while ptr[u] + c < len(s) and (s[ptr[u] + c] is None or lim_of(s[ptr[u] + c]) <= k):
                c += 1
            cnt.append(c)
        mx = max(cnt)
        steps += mx  # the kernel's sub-round loop ends when no lane can step
        for u in range(len(units)):
            ptr[u] += cnt[u]
    return steps


def sched_b(units, S):
    srcs = [word_src(p) for p in units]
    ptr = [0] * len(units)
    blk = [0] * len(units)
    steps = 0
    while any(ptr[u] < len(s) for u, s in enumerate(srcs)):
        mx = 0
        for u, s in enumerate(srcs):
            c = 0
            while c < S and ptr[u] < len(s) and (s[ptr[u]] is None or lim_of(s[ptr[u]]) <= blk[u]):
                ptr[u] += 1
                c += 1
            mx = max(mx, c)
            if ptr[u] < len(s) and s[ptr[u]] is not None and lim_of(s[ptr[u]]) > blk[u]:
                blk[u] += 1
        steps += mx
    return steps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for thr, name in ((26, "p=0.1"), (128, "p=0.5"), (230, "p=0.9")):
        data = oracle.generate(n, 4096, seed=0xC0DE0003, zero_thresh=thr)
        packed = [oracle.pack(data[i * 4096:(i + 1) * 4096].tobytes())[1] for i in range(n)]
        wa = wb = 0
        for w0 in range(0, n, 64):
            g = packed[w0:w0 + 64]
            wa += sched_a(g, S)
            wb += sched_b(g, S)
        words = n * 512
        print(f"{name}: A eff {words / (wa * 64):.3f} ({wa * 64 / n:.0f} lane-steps/unit), "
              f"B eff {words / (wb * 64):.3f} ({wb * 64 / n:.0f})")


if __name__ == "__main__" and len(sys.argv) <= 3 and sys.argv[1:2] != ["D"]:
    main()


def sched_c(units, S, R, G=16):
    """C: a ring of R 16-B pieces per lane, advanced piece by piece at every sub-round boundary
    (as far as the lane has consumed); sources below 16 q + 16 R - 10 (q = the ring's first piece)."""
    srcs = [word_src(p) for p in units]
    ptr = [0] * len(units)
    q = [0] * len(units)
    steps = 0
    while any(ptr[u] < len(s) for u, s in enumerate(srcs)):
        mx = 0
        for u, s in enumerate(srcs):
            c = 0
            while c < S and ptr[u] < len(s) and (s[ptr[u]] is None or s[ptr[u]] < G * q[u] + 16 * R - 10):
                ptr[u] += 1
                c += 1
            mx = max(mx, c)
            nxt = next((x for x in s[ptr[u]:] if x is not None), None)
            if nxt is not None:
                q[u] = max(q[u], nxt // G)  # granules below the next source are consumed
        steps += mx
    return steps


if __name__ == "__main__" and len(sys.argv) > 3:
    n, S, R = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    G = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    for thr, name in ((26, "p=0.1"), (128, "p=0.5"), (230, "p=0.9")):
        data = oracle.generate(n, 4096, seed=0xC0DE0003, zero_thresh=thr)
        packed = [oracle.pack(data[i * 4096:(i + 1) * 4096].tobytes())[1] for i in range(n)]
        wc = sum(sched_c(packed[w0:w0 + 64], S, R, G) for w0 in range(0, n, 64))
        print(f"{name}: C(S={S}, R={R}, G={G}) eff {n * 512 / (wc * 64):.3f} ({wc * 64 / n:.0f} lane-steps/unit)")


def sched_d(units, S, R=4):
    """D: C with block-aligned landing: a unit's next aligned 64-B block is requested (one quad
    load) once the ring holds all of the previous landing block, and may enter the ring from the
    next boundary on; the ring moves piece by piece over whatever has landed."""
    srcs = [word_src(p) for p in units]
    ptr = [0] * len(units)
    q = [0] * len(units)
    landed = [2] * len(units)   # blocks [0, landed) are available to the ring (0: ring, 1: landing)
    pending = [False] * len(units)
    steps = 0
    while any(ptr[u] < len(s) for u, s in enumerate(srcs)):
        mx = 0
        for u, s in enumerate(srcs):
            c = 0
            while c < S and ptr[u] < len(s) and (s[ptr[u]] is None or s[ptr[u]] < 16 * q[u] + 16 * R - 10):
                ptr[u] += 1
                c += 1
            mx = max(mx, c)
        steps += mx
        for u, s in enumerate(srcs):  # boundary
            if pending[u]:
                landed[u] += 1
                pending[u] = False
            nxt = next((x for x in s[ptr[u]:] if x is not None), None)
            if nxt is not None:
                q[u] = max(q[u], min(nxt // 16, 4 * landed[u] - R))
            if q[u] >= 4 * (landed[u] - 1) and not pending[u]:
                pending[u] = True  # the landing block moved in whole: request the next one
    return steps


if __name__ == "__main__" and len(sys.argv) == 2 and sys.argv[1] == "D":
    n = 256
    for thr, name in ((26, "p=0.1"), (128, "p=0.5"), (230, "p=0.9")):
        data = oracle.generate(n, 4096, seed=0xC0DE0003, zero_thresh=thr)
        packed = [oracle.pack(data[i * 4096:(i + 1) * 4096].tobytes())[1] for i in range(n)]
        wd = sum(sched_d(packed[w0:w0 + 64], 8) for w0 in range(0, n, 64))
        print(f"{name}: D eff {n * 512 / (wd * 64):.3f} ({wd * 64 / n:.0f} lane-steps/unit)")
