"""Dev model (round 5): host restatement of decode_words_kernel's per-lane logic, checked against
the oracle (message.zig:88-191 restated in oracle/packed_oracle.c).

Per unit (one lane): aligned-space positions pos in [s, s + P), rounds k = 0 .. maxr with the ring
window [64k - 12, 64k + 64) (bytes outside the unit read as whatever the clamped loads left:
modelled as random garbage), sources of round k below lim = min(64k + 52, end), one word per step:
record (r == 0), zero word (zrem > 0), literal word (lrem > 0). Checks the words, the EOF status
and out_len on random units of every density, truncations and the adversarial corpus.
Usage: python3 scripts/dev/sim_words.py [n]
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle  # noqa: E402

DEAD = 0xFFFFFFFF


def popc(x):
    return bin(x).count("1")


def sim_unit(p: bytes, s: int, rng):
    P = len(p)
    end = s + P
    maxr = (end + 63) >> 6
    # aligned-space byte view: positions < s and >= end are garbage (the ring's clamped loads)
    garbage = bytes(rng.randrange(256) for _ in range(64 * (maxr + 2) + 64))

    def byte_at(q):
        if s <= q < end:
            return p[q - s]
        return garbage[q % len(garbage)]

    pos, run, rsel, apos = (s if P else DEAD), 0, 0, (s if P else DEAD)
    words = []
    for k in range(maxr + 1):
        base = 64 * k - 12
        lim = min(64 * k + 52, end)
        while apos < lim:
            o = min(max(pos - base, 0), 64)
            q = base + o  # the ring's byte o
            assert 0 <= o <= 64 and (o & ~3) + 12 <= 76  # every read inside the 76-B ring
            t, b1, c9 = byte_at(q), byte_at(q + 1), byte_at(q + 9)
            inrec = run == 0
            tz, tf = t == 0, t == 0xFF
            ln = popc(t) + 1 + (1 if (tz or tf) else 0)
            cnt = b1 if tz else (c9 if tf else 0)
            tsel = t if inrec else rsel
            po = o + (1 if inrec else 0)
            pay = [byte_at(base + po + i) for i in range(8)]
            if tsel == 0:
                word = bytes(8)
            elif tsel == 0xFF:
                word = bytes(pay)
            else:
                it = iter(pay)
                word = bytes(next(it) if (tsel >> i) & 1 else 0 for i in range(8))
            pos += ln if inrec else (rsel & 8)
            run = cnt if inrec else run - 1
            rsel = (0xFF if tf else 0) if inrec else rsel
            apos = 0 if (run != 0 and rsel == 0) else pos
            words.append(word)
    eof = P > 0 and (pos != end or run != 0)
    return ("EOF", b"") if eof else ("OK", b"".join(words))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rng = random.Random(5)
    cases = []
    for i in range(n):
        nw = rng.choice([0, 1, 2, 7, 31, 64, 200, 512, 700])
        pz = rng.choice([0.0, 0.1, 0.5, 0.9, 1.0])
        d = bytes((0 if rng.random() < pz else rng.randrange(1, 256)) for _ in range(8 * nw))
        st, pk = oracle.pack(d)
        assert st == 0
        cases.append(pk)
        if len(pk) > 1:
            cases.append(pk[:rng.randrange(1, len(pk))])  # truncated
    corpus = [b"", b"\x01", b"\x00", b"\xff", b"\xff\x01\x02\x03\x04", bytes([0xFF] + list(range(1, 9))),
              bytes([0xFF] + list(range(1, 9)) + [1]), bytes([0xFF] + list(range(1, 9)) + [1, 0xAA, 0xBB]),
              bytes([0xFF] + list(range(1, 9)) + [0xFF]), b"\xfe\x01\x02", b"\x80", b"\x00\x00\x01", b"\xff" * 10,
              b"\x03\xaa", b"\x00\x00", b"\x00\xff", bytes([0xFF] + list(range(1, 9)) + [0]), b"\x00\x00\x00\x00",
              b"\x00\x03", bytes([0, 1, 0xFF] + list(range(1, 9)) + [0]), b"\x10\x01\x00\x00", b"\x00\x01",
              b"\x00\xff" * 40, bytes([0xFF] + [7] * 8 + [255] + [9] * 2040)]
    cases += corpus
    bad = 0
    for pk in cases:
        ost, out = oracle.unpack(pk)
        want = ("OK", out) if ost == 0 else ("EOF", b"")
        for s in (0, 5, 15):
            got = sim_unit(pk, s, rng)
            if got != want:
                bad += 1
                if bad < 5:
                    print("MISMATCH", pk[:40].hex(), len(pk), s, got[0], len(got[1]), want[0], len(want[1]))
    print(f"{len(cases)} units x 3 alignments: {bad} mismatches")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
