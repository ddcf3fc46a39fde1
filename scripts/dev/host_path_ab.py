#!/usr/bin/env python3
"""Dev-only: bench.host_path (PCIe-inclusive decode / encode of 64K x 4 KiB units, pinned host
buffers) over chunk / stream counts, twice each, same process."""
import json, os, sys, types
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
import bench

args = types.SimpleNamespace(unit_bytes=4096, seed=0xC0DE0003, zero_thresh=128)
dev = torch.device("cuda", 0)
for rep in range(2):
    for chunks, ns in ((8, 2), (16, 3), (32, 4), (64, 4)):
        r = bench.host_path(args, dev, n_units=1 << 16, chunks=chunks, nstreams=ns)
        print(json.dumps({k: r[k] for k in ("chunks", "streams", "decode_GiB_s", "encode_GiB_s", "bit_exact_roundtrip")}),
              flush=True)
