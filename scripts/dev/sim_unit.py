#!/usr/bin/env python3
"""CPU simulation of decode_unit_kernel's chain resolution (dev diagnostic, not a test).

For random units of a zero-byte density it reports how many walks the lanes need
(1 = the entry maps were right everywhere) and the per-lane record counts.
"""
import collections
import random
import sys

sys.path.insert(0, "tests")
import pyref  # noqa: E402


def gen(p, nbytes, rng):
    return bytes(0 if rng.random() < p else rng.randrange(1, 256) for _ in range(nbytes))


def rec_len(pk, x):
    t = pk[x]
    if t == 0:
        return 2
    if t == 0xFF:
        return 10 + 8 * (pk[x + 9] if x + 9 < len(pk) else 0)
    return 1 + bin(t).count("1")


def entry_map(pk, rs, re, mode):
    # states for entries 0..7 after bytes [rs, re); FF -> absorbing 'X'
    st = list(range(8))
    for x in range(rs, re):
        t = pk[x] if x < len(pk) else 0
        for e in range(8):
            d = st[e]
            if d == "X":
                continue
            if d == 0:
                if t == 0xFF:
                    st[e] = "X" if mode != "ff16" else None
                    if mode == "ff16":
                        c = pk[x + 9] if x + 9 < len(pk) else 0
                        st[e] = 9 + 8 * c
                else:
                    st[e] = max(bin(t).count("1"), 1)
            else:
                st[e] = d - 1
    return st


def sim(p, units=200, seed=1, mode="x"):
    rng = random.Random(seed)
    walks = collections.Counter()
    maxrec = []
    for _ in range(units):
        pk = pyref.pack(gen(p, 4096, rng)) + bytes(32)
        P = len(pk) - 32
        np_ = (P + 15) // 16
        L = (np_ + 63) // 64
        lanes = []
        for l in range(64):
            q0 = min(l * L, np_)
            q1 = min(q0 + L, np_)
            if q0 >= np_:
                break
            lanes.append((16 * q0, min(16 * q1, P)))
        maps = []
        for (rs, re) in lanes:
            st = entry_map(pk, rs, rs + 16 * L, mode)
            nx = [v for v in st if v != "X" and v is not None and v < 8]
            R = nx[0] if nx else 0
            maps.append([v if (v != "X" and v is not None and v < 8) else R for v in st])
        # scan
        entries = [0]
        e = 0
        for k in range(1, len(lanes)):
            e = maps[k - 1][e]
            entries.append(lanes[k][0] + e)

        def walk(k, pos):
            rs, je = lanes[k]
            n = 0
            while pos < je:
                ln = rec_len(pk, pos)
                if pos + ln > P:
                    return 1 << 40, n
                pos += ln
                n += 1
            return pos, n

        ex = [walk(k, entries[k])[0] for k in range(len(lanes))]
        nw = 1
        for _it in range(64):
            fur = 0
            redo = []
            for k in range(len(lanes)):
                if k > 0 and fur != entries[k]:
                    redo.append(k)
                fur = max(fur, ex[k])
            if not redo:
                break
            nw += 1
            fur = 0
            want = []
            for k in range(len(lanes)):
                want.append(fur)
                fur = max(fur, ex[k])
            for k in redo:
                entries[k] = want[k]
                ex[k] = walk(k, entries[k])[0]
        walks[nw] += 1
        maxrec.append(max(walk(k, entries[k])[1] for k in range(len(lanes))))
    return walks, sum(maxrec) / len(maxrec)


if __name__ == "__main__":
    for p in (0.5, 0.1, 0.9):
        w, mr = sim(p, units=int(sys.argv[1]) if len(sys.argv) > 1 else 100)
        print(p, dict(sorted(w.items())), "max records/lane %.1f" % mr)
