#!/usr/bin/env python3
"""Dev-only: fused framing encode (bench.message_leg) at segment shapes whose 16-B pair loads are
aligned or not, and one-segment messages (no segment map): 1 segment of 509 words, 3 segments (2 header words) of 170 words (1360 B, pairs 16-B aligned) or 169
words, and 4 segments (3 header words) of 127 / 126 words (pairs 8 mod 16). Twice each."""
import json, os, sys, types
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
import bench

args = types.SimpleNamespace(units=1 << 20, zero_thresh=128)
dev = torch.device("cuda", 0)
for rep in range(2):
    for segs, sw in ((1, 509), (3, 170), (4, 127)):
        r = bench.message_leg(args, dev, segs=segs, seg_words=sw)
        print(json.dumps({"segs": segs, "seg_words": sw, "framed_bytes": r["framed_bytes"],
                          "fused_encode_ms": r["fused_encode_ms"], "encode_frac": r["encode_frac"],
                          "bit_exact": r["bit_exact"]}), flush=True)
        torch.cuda.empty_cache()
