#!/usr/bin/env python3
"""Dev: config C5 with the Pareto sizes capped at CAP bytes (tail-latency experiment)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np
import torch
import bench

cap = int(sys.argv[1])
orig = bench.pareto_sizes
bench.pareto_sizes = lambda n, seed=0xC0DE0005: np.minimum(orig(n, seed), cap)
class A: zero_thresh = 128
print(json.dumps({"cap": cap, **bench.skewed_leg(A(), torch.device("cuda", 0))}))
