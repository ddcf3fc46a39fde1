"""Dev model (round 5): the index walk with two records per step (decode_index_kernel, !kStop)
against the one-record walk, per unit: the record starts (piece records' bits), the words per
piece, the end position and the EOF outcome must be identical. Positions in aligned space,
rounds of 64 B: round k walks the tags in [64k - 16, 64k + 48) below the unit's end.
Usage: python3 scripts/dev/sim_pair.py [n]"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle  # noqa: E402


def popc(x):
    return bin(x).count("1")


def walk(p, s, pair):
    end = s + len(p)
    byte = lambda q: p[q - s] if s <= q < end else random.randrange(256)  # noqa: E731
    nr = (end + 63) >> 6
    pos, starts, words, eof = s, [], {}, False
    for k in range(nr + 1):
        lim = min(64 * k + 48, end)
        while pos < lim and not eof:
            t, b1, c9 = byte(pos), byte(pos + 1), byte(pos + 9)
            z, f = t == 0, t == 0xFF
            ln = 1 + popc(t) + (1 if (z or f) else 0) + (8 * c9 if f else 0)
            if pos + ln > end:
                eof = True
                break
            starts.append(pos)
            words[pos >> 4] = words.get(pos >> 4, 0) + 1 + (b1 if z else 0) + (c9 if f else 0)
            p1 = pos + ln
            if pair and not f:
                t2, b2 = byte(p1), byte(p1 + 1)
                ln2 = 1 + popc(t2) + (1 if t2 == 0 else 0)
                assert ln <= 8
                if t2 != 0xFF and p1 < lim and p1 + ln2 <= end:
                    starts.append(p1)
                    words[p1 >> 4] = words.get(p1 >> 4, 0) + 1 + (b2 if t2 == 0 else 0)
                    p1 += ln2
            pos = p1
    return starts, words, pos, eof


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    rng = random.Random(7)
    bad = 0
    for i in range(n):
        nw = rng.choice([1, 2, 7, 64, 200, 512, 900])
        pz = rng.choice([0.0, 0.1, 0.5, 0.9, 1.0])
        d = bytes((0 if rng.random() < pz else rng.randrange(1, 256)) for _ in range(8 * nw))
        st, pk = oracle.pack(d)
        cases = [pk, pk[:rng.randrange(1, len(pk))]] if len(pk) > 1 else [pk]
        for c in cases:
            for s in (0, 3, 8, 15):
                a, b = walk(c, s, False), walk(c, s, True)
                if a != b:
                    bad += 1
    print(f"{n} units: {bad} mismatches")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
