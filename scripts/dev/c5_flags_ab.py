#!/usr/bin/env python3
"""Dev-only: the C5 leg (bench.skewed_leg) with and without LAUNCH_MID_SIDE_STREAM (mid units on a
second side stream beside the small-unit kernels, encode and decode), alternating, same process."""
import json, os, sys, types
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
import bench
import capnp_packed as cp

args = types.SimpleNamespace(zero_thresh=128, seed=0xC0DE0003, unit_bytes=4096)
dev = torch.device("cuda", 0)
for r in range(3):
    for flags in (0, cp.LAUNCH_MID_SIDE_STREAM):
        with cp.launch_flags(flags):
            res = bench.skewed_leg(args, dev)
        print(json.dumps({"flags": flags, "encode_ms": res["encode_ms"], "decode_ms": res["decode_ms"],
                          "GiB_s": res["GiB_s"], "bit_exact": res["bit_exact_roundtrip"]}), flush=True)
