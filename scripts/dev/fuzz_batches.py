#!/usr/bin/env python3
"""Dev (round 6): randomized batch fuzzing of the shipped kernels against the oracle, for a wall
budget. Each round builds a batch of mixed units (small / mid / long sizes, densities 0..1,
16-B or 8-B mod 16 starts, empty and odd-size units), encodes it into slots of random slack
(some too small), checks every status and byte against oracle.pack_batch, then decodes the
packed units (some truncated or corrupted, some slots short) under auto / twopass / words and
checks statuses, lengths and bytes against oracle.unpack_batch. Prints one JSON line.
Usage: python3 scripts/dev/fuzz_batches.py [--seconds 240] [--units 20000]"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "capnp-zig_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))

import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402
import oracle  # noqa: E402

DEV = torch.device("cuda", 0)
BIG = False


def t64(a):
    return torch.from_numpy(np.asarray(a, dtype=np.int64)).to(DEV)


def layout(sizes, rng, mods=(0, 8)):
    offs, pos = np.zeros(len(sizes), np.int64), 0
    for i, s in enumerate(sizes):
        pos = (pos + 15) // 16 * 16 + int(rng.choice(mods))
        offs[i] = pos
        pos += int(s)
    return offs, pos


def one_round(rng, n, stats):
    kind = rng.integers(0, 10, n)
    words = np.where(kind < 5, rng.integers(0, 65, n),
                     np.where(kind < 9, rng.integers(65, 513, n), rng.integers(513, 4097, n)))
    if BIG:  # C5's tail: 0.5% of units of 64 KiB .. 256 KiB (the huge class and long windows)
        huge = rng.random(n) < 0.005
        words[huge] = rng.integers(8192, 32769, int(huge.sum()))
    words[rng.random(n) < 0.3] = 512
    sizes = words * 8
    odd = rng.random(n) < 0.005
    sizes[odd] += rng.integers(1, 8, int(odd.sum()))
    dens = rng.choice([0.0, 0.05, 0.1, 0.5, 0.9, 0.95, 1.0], n)
    offs, total = layout(sizes, rng)
    host = np.zeros(total + 64, np.uint8)
    for i in range(n):
        s = int(sizes[i])
        if s == 0:
            continue
        v = rng.integers(1, 256, s, dtype=np.uint8)
        v[rng.random(s) < dens[i]] = 0
        if rng.random() < 0.05:  # long zero / literal stretches
            a = int(rng.integers(0, s))
            v[a:a + int(rng.integers(0, 4096))] = 0 if rng.random() < 0.5 else 7
        host[offs[i]:offs[i] + s] = v
    # encode slots: the bound, +slack, or short
    bound = np.array([cp.encode_bound(int(s)) for s in sizes], np.int64)
    caps = bound + rng.integers(0, 17, n)
    short = rng.random(n) < 0.02
    caps[short] = (bound[short] * rng.random(int(short.sum())) * 0.6).astype(np.int64)
    pk_off = np.zeros(n + 1, np.int64)
    pk_off[1:] = np.cumsum((caps + 15) // 16 * 16)
    d_in = torch.from_numpy(host).to(DEV)
    d_pk = torch.full((int(pk_off[-1]) + 64,), 0xEE, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int64, device=DEV)
    pst = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    cp.encode_batch(d_in, t64(offs), t64(sizes), d_pk, t64(pk_off[:-1]), t64(caps), plen, pst)
    torch.cuda.synchronize()
    # oracle (slot-sized batches with the same caps)
    in_off_o = np.zeros(n + 1, np.uint64)
    in_off_o[1:] = np.cumsum(sizes)
    flat = np.concatenate([host[offs[i]:offs[i] + int(sizes[i])] for i in range(n)]) if n else np.zeros(0, np.uint8)
    o_off = np.zeros(n + 1, np.uint64)
    o_off[1:] = np.cumsum(caps)
    r, r_len, r_st = oracle.pack_batch(flat, in_off_o, o_off)
    g_st, g_len, pk = pst.cpu().numpy(), plen.cpu().numpy(), d_pk.cpu().numpy()
    bad = []
    for i in range(n):
        if g_st[i] != r_st[i] or (r_st[i] == 0 and g_len[i] != r_len[i]):
            bad.append(("enc-status", i, int(sizes[i]), int(g_st[i]), int(r_st[i])))
            continue
        if r_st[i] == 0:
            a, b = int(pk_off[i]), int(o_off[i])
            if not np.array_equal(pk[a:a + int(g_len[i])], r[b:b + int(r_len[i])]):
                bad.append(("enc-bytes", i, int(sizes[i])))
            elif int(caps[i]) > int(g_len[i]) and pk[a + int(g_len[i]):a + int(caps[i])].max(initial=0xEE) != 0xEE:
                bad.append(("enc-past-len", i, int(sizes[i])))
    stats["enc_units"] += n
    # decode: OK units' packed bytes, some truncated / corrupted, slots exact / short
    ok = np.where(r_st == 0)[0]
    units, dcaps = [], []
    for i in ok:
        b = int(o_off[i])
        p = r[b:b + int(r_len[i])].copy()
        x = rng.random()
        if x < 0.03 and len(p):
            p = p[:int(rng.integers(0, len(p)))]
        elif x < 0.06 and len(p):
            p[int(rng.integers(0, len(p)))] = int(rng.integers(0, 256))
        units.append(p)
        c = int(sizes[i]) if rng.random() > 0.03 else max(int(sizes[i]) - 8 * int(rng.integers(1, 4)), 0)
        dcaps.append(c)
    m = len(units)
    p_offs, ptot = layout([len(u) for u in units], rng, mods=tuple(range(16)))
    phost = np.zeros(ptot + 64, np.uint8)
    for o, u in zip(p_offs, units):
        phost[o:o + len(u)] = u
    d_p = torch.from_numpy(phost).to(DEV)
    dcaps = np.array(dcaps, np.int64)
    u_off = np.zeros(m + 1, np.int64)
    u_off[1:] = np.cumsum((dcaps + 15) // 16 * 16 + 16)
    pin_off = np.zeros(m + 1, np.uint64)
    pin_off[1:] = np.cumsum([len(u) for u in units])
    pflat = np.concatenate(units) if m else np.zeros(0, np.uint8)
    uo_off = np.zeros(m + 1, np.uint64)
    uo_off[1:] = np.cumsum(dcaps)
    e, e_len, e_st = oracle.unpack_batch(pflat, pin_off, uo_off)
    for dec in ("auto", "twopass", "words"):
        if not cp.decoder_available(dec):
            continue
        with cp.decoder(dec):
            d_u = torch.full((int(u_off[-1]) + 64,), 0xEE, dtype=torch.uint8, device=DEV)
            ulen = torch.zeros(m, dtype=torch.int64, device=DEV)
            ust = torch.full((m,), -1, dtype=torch.int32, device=DEV)
            cp.decode_batch(d_p, t64(p_offs), t64([len(u) for u in units]), d_u, t64(u_off[:-1]), t64(dcaps),
                            ulen, ust)
            torch.cuda.synchronize()
        gs, gl, gu = ust.cpu().numpy(), ulen.cpu().numpy(), d_u.cpu().numpy()
        for j in range(m):
            a = int(u_off[j])
            if gs[j] != e_st[j] or (e_st[j] == 0 and gl[j] != e_len[j]):
                bad.append((f"dec-{dec}-status", j, len(units[j]), int(gs[j]), int(e_st[j])))
            elif e_st[j] == 0 and not np.array_equal(gu[a:a + int(gl[j])], e[int(uo_off[j]):int(uo_off[j]) + int(e_len[j])]):
                bad.append((f"dec-{dec}-bytes", j, len(units[j])))
            if gu[a + int(dcaps[j]):a + int(dcaps[j]) + 16].min(initial=0xEE) != 0xEE:
                bad.append((f"dec-{dec}-past-cap", j, len(units[j])))
        stats["dec_units"] += m
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--units", type=int, default=20000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--big", action="store_true", help="add units of 64-256 KiB")
    a = ap.parse_args()
    global BIG
    BIG = a.big
    rng = np.random.default_rng(a.seed)
    stats = {"rounds": 0, "enc_units": 0, "dec_units": 0}
    bad, t0 = [], time.time()
    while time.time() - t0 < a.seconds:
        bad += one_round(rng, a.units, stats)
        stats["rounds"] += 1
        print(json.dumps({"progress": stats, "bad": len(bad), "t": round(time.time() - t0, 1)}), flush=True)
        if len(bad) > 50:
            break
    print(json.dumps({"stats": stats, "bad": bad[:50]}))


if __name__ == "__main__":
    main()
