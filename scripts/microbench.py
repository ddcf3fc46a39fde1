#!/usr/bin/env python3
"""Component timings for the packed codec kernels (diagnostics, not the bench).

Times, on one GPU with HIP events on the launch stream (median of --reps):
  encode (slots), encoded-size only, decode (from slots), decoded-size only,
  and torch copy / fill kernels of the same byte counts as bandwidth references.
"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "capnp-zig_amd"))

import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402


def timeit(fn, reps):
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--units", type=int, default=1 << 20)
    ap.add_argument("--unit-bytes", type=int, default=4096)
    ap.add_argument("--zero-thresh", type=int, default=128)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--only", default="")
    ap.add_argument("--pk-stride", type=int, default=0, help="packed slot stride (default encode_bound)")
    ap.add_argument("--dense", action="store_true", help="decode from a dense packed stream")
    ap.add_argument("--no-store", action="store_true", help="decode with zero output capacity (walk only, no stores)")
    ap.add_argument("--decoder", default="", help="mid-unit decoder (capnp_packed_set_decoder name)")
    a = ap.parse_args()
    if a.decoder:
        cp.set_decoder(a.decoder)
    n, ub = a.units, a.unit_bytes
    dev = torch.device("cuda", 0)
    d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=a.zero_thresh, device=dev)
    in_off, in_len = cp.uniform_layout(n, ub, device=dev)
    slot = a.pk_stride or cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    pk_cap.fill_(cp.encode_bound(ub))
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.zeros(n, dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
    ulen = torch.zeros(n, dtype=torch.int64, device=dev)
    ust = torch.zeros(n, dtype=torch.int32, device=dev)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    torch.cuda.synchronize()
    P = int(plen.sum().item())
    if a.dense:  # repack into a dense stream (test plumbing, untimed)
        off = cp.lengths_to_offsets(plen)
        dense = torch.empty(P + 16, dtype=torch.uint8, device=dev)
        rows = d_pk.view(n, slot)
        keep = torch.arange(slot, device=dev).unsqueeze(0) < plen.unsqueeze(1)
        dense[:P] = rows[keep]
        d_pk, pk_off = dense, off[:-1].contiguous()
    U = n * ub
    ocap = torch.zeros_like(in_len) if a.no_store else in_len
    res = {"units": n, "unit_bytes": ub, "P": P, "U": U}
    cases = {
        "encode": lambda: cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst),
        "encoded_size": lambda: cp.encoded_size_batch(d_in, in_off, in_len, plen, pst),
        "decode": lambda: cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, ocap, ulen, ust),
        "decoded_size": lambda: cp.decoded_size_batch(d_pk, pk_off, plen, ulen, ust),
        "copy_U": lambda: d_out.copy_(d_in),
        "fill_U": lambda: d_out.fill_(1),
    }
    for name, fn in cases.items():
        if a.only and name not in a.only.split(","):
            continue
        fn()
        ms = timeit(fn, a.reps)
        res[name + "_ms"] = round(ms, 4)
    res["copy_U_GBps"] = round(2 * U / (res.get("copy_U_ms", 1e9) * 1e-3) / 1e9, 1)
    res["fill_U_GBps"] = round(U / (res.get("fill_U_ms", 1e9) * 1e-3) / 1e9, 1)
    ok = bool((ust == 0).all().item()) if ("decode_ms" in res and not a.no_store) else None
    if "decoded_size_ms" in res:
        cp.decoded_size_batch(d_pk, pk_off, plen, ulen, ust)
        torch.cuda.synchronize()
        res["size_ok"] = bool(torch.equal(ulen, in_len)) and bool((ust == 0).all().item())
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
    torch.cuda.synchronize()
    res["roundtrip_ok"] = bool(torch.equal(d_out, d_in)) and ok is not False
    print(json.dumps(res))


if __name__ == "__main__":
    main()
