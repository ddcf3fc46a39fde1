"""Dev model (round 5): a lane-per-unit streaming decoder that emits ONE output word per step.

A wave owns 64 units; round k stages each unit's packed bytes [64k, 64k + 64) next to the last 16 B
of round k-1 (an 80-B ring), and every lane emits the words whose source starts in
[64k - 16, 64k + 48): a record's first word (mixed tag, FF head, 00 head), one literal word of an FF
body, or one zero word of a zero run. A round is cut into sub-rounds of S steps (after each, the
sub-round's words are stored), so a round costs ceil(max_u words_u / S) sub-rounds. Zero runs with
more than Z extra words go to a wave job (the lane emits the first word and skips the rest).
Prints the step efficiency (words / (64 x S x sub-rounds)) per density.
Usage: python3 scripts/dev/sim_lane_words.py [units] [S] [Z]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle  # noqa: E402


def word_sources(p, Z):
    """(source byte position, kind) per emitted word; kind 0 record head, 1 literal, 2 zero word."""
    out = []
    i, n = 0, len(p)
    while i < n:
        t = p[i]
        if t == 0:
            c = p[i + 1]
            out.append((i, 0))
            for _ in range(min(c, Z) if c <= Z else 0):
                out.append((i, 2))  # zero words emitted at the head's round
            i += 2
        elif t == 0xFF:
            c = p[i + 9]
            out.append((i, 0))
            for j in range(c):
                out.append((i + 10 + 8 * j, 1))
            i += 10 + 8 * c
        else:
            out.append((i, 0))
            i += 1 + bin(t).count("1")
    return out


def round_of(pos):
    # round k takes sources in [64k - 16, 64k + 48)
    return (pos + 16) // 64


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    Z = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    for thr, name in ((26, "p=0.1"), (128, "p=0.5"), (230, "p=0.9")):
        data = oracle.generate(n, 4096, seed=0xC0DE0003, zero_thresh=thr)
        packed = [oracle.pack(data[i * 4096:(i + 1) * 4096].tobytes())[1] for i in range(n)]
        words_total, sub_total, steps_total, rounds_total = 0, 0, 0, 0
        for w0 in range(0, n, 64):
            grp = packed[w0:w0 + 64]
            per = []
            R = 0
            for p in grp:
                src = word_sources(bytes(p) + bytes(16), Z)
                cnt = {}
                for pos, _ in src:
                    if pos >= len(p):
                        continue
                    k = round_of(pos)
                    cnt[k] = cnt.get(k, 0) + 1
                per.append(cnt)
                R = max(R, (len(p) + 16 + 63) // 64 + 1)
            for k in range(R):
                ws = [c.get(k, 0) for c in per]
                mx = max(ws)
                words_total += sum(ws)
                sub_total += (mx + S - 1) // S
                steps_total += mx
            rounds_total += R
        nw = n
        print(f"{name}: words/unit {words_total / nw:.0f} | rounds/wave {rounds_total / ((n + 63) // 64):.1f} | "
              f"steps/wave-unit {steps_total / nw * 64 / 64:.0f} (lockstep eff {words_total / (64 * steps_total) * 64 / 64:.2f}) | "
              f"sub-rounds/round {sub_total / rounds_total:.2f} | eff with S={S}: {words_total / (S * sub_total * 64) * 64 / 64:.2f}")


if __name__ == "__main__":
    main()
