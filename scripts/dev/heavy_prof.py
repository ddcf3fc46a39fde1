#!/usr/bin/env python3
"""Dev (round 6): the headline decode with and without 64 expansion-heavy units (00 FF chains),
for a kernel trace (rocprofv3 --kernel-trace --stats)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "capnp-zig_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402

n, ub = 1 << 20, 4096
dev = torch.device("cuda", 0)
d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=128, device=dev)
in_off, in_len = cp.uniform_layout(n, ub, device=dev)
slot = cp.encode_bound(ub)
pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
plen = torch.empty(n, dtype=torch.int64, device=dev)
pst = torch.empty(n, dtype=torch.int32, device=dev)
cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
ulen = torch.empty(n, dtype=torch.int64, device=dev)
ust = torch.empty(n, dtype=torch.int32, device=dev)
mode = sys.argv[1] if len(sys.argv) > 1 else "heavy"
if mode == "heavy":
    rng = np.random.default_rng(0xE4)
    heavy = np.sort(rng.choice(n, 64, replace=False))
    chain = bytes([0, 0xFF]) * 1250
    hb = torch.from_numpy(np.frombuffer(chain, dtype=np.uint8).copy()).to(dev)
    for u in heavy.tolist():
        d_pk[u * slot:u * slot + len(chain)] = hb
        plen[u] = len(chain)
torch.cuda.synchronize()
for _ in range(6):
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
torch.cuda.synchronize()
print(mode, "statuses", np.unique(ust.cpu().numpy(), return_counts=True))
