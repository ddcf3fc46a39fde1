"""Dev model (round 5): statistics of lane-block record chains for a wave-per-unit decoder.

For Zig-packed 4 KiB units at p = 0.1 / 0.5 / 0.9 (the bench's generator), cut each unit's packed
bytes into 64 lane blocks and measure what a speculative per-lane walk would cost:
  - records per lane (mean, and the wave's max: what a lockstep loop runs to);
  - spec walk started W bytes before the block (W = 0: at the block start): does its chain contain
    the true entry (the first true record start >= block start)?  If not, how many true records
    until the two chains meet (the re-walk a verify round costs);
  - verify rounds with neighbour propagation.
Usage: python3 scripts/dev/sim_spec.py [units]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import oracle  # noqa: E402


def rec_len(p, i):
    t = p[i]
    if t == 0:
        return 2
    if t == 0xFF:
        c = p[i + 9] if i + 9 < len(p) else 0
        return 10 + 8 * c
    return 1 + bin(t).count("1")


def chain(p, start, stop):
    """Record starts from start while < stop (positions may run past len(p))."""
    out = []
    i = start
    while i < stop:
        out.append(i)
        i += rec_len(p, i)
    return out, i


def unit_stats(p, W, lanes=64, piece=16):
    P = len(p)
    np_ = (P + piece - 1) // piece
    L = (np_ + lanes - 1) // lanes
    B = L * piece
    pad = bytes(p) + bytes(2100)  # reads past the end see zeros
    true, _ = chain(pad, 0, P)
    tset = set(true)
    tarr = np.array(true + [1 << 30])
    recs, bad, merge, ff_far = [], 0, [], 0
    ok = []
    for l in range(lanes):
        s, e = l * B, min((l + 1) * B, P)
        if s >= P:
            break
        E = int(tarr[np.searchsorted(tarr, s)])
        nrec = int(np.searchsorted(tarr, e) - np.searchsorted(tarr, s))
        recs.append(nrec)
        if E >= e:
            ff_far += 1  # covered by an FF body: pass-through lane
            ok.append(True)
            continue
        spec, _ = chain(pad, max(0, s - W), e)
        sset = set(spec)
        good = E in sset
        ok.append(good)
        if not good:
            bad += 1
            k = 0
            q = E
            while q < e and q not in sset:
                q += rec_len(pad, q)
                k += 1
            merge.append(k)
    # verify rounds: lane l is fixed in the round after all its predecessors are; a good lane
    # whose predecessor chain is right needs no round of its own
    rounds, run = 0, 0
    for g in ok:
        run = 0 if g else run + 1
        rounds = max(rounds, run)
    return recs, bad, merge, ff_far, rounds, B


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    for thr, name in ((26, "p=0.1"), (128, "p=0.5"), (230, "p=0.9")):
        data = oracle.generate(n, 4096, seed=0xC0DE0003, zero_thresh=thr)
        packed = [oracle.pack(data[i * 4096:(i + 1) * 4096].tobytes())[1] for i in range(n)]
        Ps = [len(x) for x in packed]
        print(f"{name}: P mean {np.mean(Ps):.0f}")
        for W in (0, 8, 16, 24):
            R, Bad, M, FF, RD, Bs = [], 0, [], 0, [], []
            mx = []
            for p in packed:
                recs, bad, merge, ff, rounds, B = unit_stats(p, W)
                R += recs
                mx.append(max(recs))
                Bad += bad
                M += merge
                FF += ff
                RD.append(rounds)
                Bs.append(B)
            nl = len(R)
            print(f"  W={W:2d} B={np.mean(Bs):.0f} recs/lane mean {np.mean(R):.1f} wave-max {np.mean(mx):.1f} | "
                  f"spec miss {Bad / nl:.3f} merge recs mean {np.mean(M) if M else 0:.2f} p99 "
                  f"{np.percentile(M, 99) if M else 0:.0f} | pass-through lanes {FF / nl:.3f} | "
                  f"verify rounds mean {np.mean(RD):.2f} max {max(RD)}")


if __name__ == "__main__":
    main()
