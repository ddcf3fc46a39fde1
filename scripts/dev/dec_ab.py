#!/usr/bin/env python3
"""Dev A/B (round 5): mid-unit decoders on the headline shape, same process, alternating.

For each density: generate 1M x 4 KiB units, encode into 5120-B slots (as bench.py), then decode
with each named decoder in turn (HIP events on the launch stream, median of --reps), and check
every decoder's output bytes, lengths and statuses against the first one's (and the input).
Usage: python3 scripts/dev/dec_ab.py [--decoders twopass,words] [--units N] [--reps 7]
"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "capnp-zig_amd"))

import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decoders", default="twopass,words")
    ap.add_argument("--units", type=int, default=1 << 20)
    ap.add_argument("--unit-bytes", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--thr", default="128,26,230")
    ap.add_argument("--dense", action="store_true", help="also decode from a dense packed stream")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, ub = a.units, a.unit_bytes
    decs = a.decoders.split(",")
    res = {}
    for thr in [int(x) for x in a.thr.split(",")]:
        d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=thr, device=dev)
        in_off, in_len = cp.uniform_layout(n, ub, device=dev)
        slot = cp.encode_bound(ub)
        pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
        d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
        plen = torch.empty(n, dtype=torch.int64, device=dev)
        pst = torch.empty(n, dtype=torch.int32, device=dev)
        cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
        torch.cuda.synchronize()
        assert int((pst != 0).sum()) == 0
        P = int(plen.sum())
        outs = {}
        times = {d: [] for d in decs}
        d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
        ulen = torch.empty(n, dtype=torch.int64, device=dev)
        ust = torch.empty(n, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream()
        for rep in range(a.reps + 1):
            for d in decs:
                with cp.decoder(d):
                    d_out.fill_(0x5A)
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record(s)
                    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
                    ev1.record(s)
                    ev1.synchronize()
                    if rep > 0:
                        times[d].append(ev0.elapsed_time(ev1))
                    if rep == 0:
                        ok = bool(torch.equal(d_out, d_in)) and int((ust != 0).sum()) == 0 and bool(
                            torch.equal(ulen, in_len))
                        outs[d] = ok
        for d in decs:
            ms = statistics.median(times[d])
            res[f"thr{thr}_{d}"] = {"ms": round(ms, 4), "frac": round((P + n * ub + 44 * n) / (ms * 1e-3) / 8e12, 4),
                                    "bit_exact": outs[d]}
        print(json.dumps({k: v for k, v in res.items() if k.startswith(f"thr{thr}_")}), flush=True)
        del d_in, d_pk, d_out
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
