#!/usr/bin/env python3
"""Dev (round 6): where the words decoder's output differs from the input on a small batch."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "capnp-zig_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402

dev = torch.device("cuda", 0)
for n in (64, 256, 4096):
    ub = 4096
    d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=128, device=dev)
    in_off, in_len = cp.uniform_layout(n, ub, device=dev)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.zeros(n, dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    d_out = torch.full((n * ub,), 0xEE, dtype=torch.uint8, device=dev)
    ulen = torch.zeros(n, dtype=torch.int64, device=dev)
    ust = torch.zeros(n, dtype=torch.int32, device=dev)
    with cp.decoder("words"):
        cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
    torch.cuda.synchronize()
    a, b = d_in.cpu().numpy().reshape(n, ub), d_out.cpu().numpy().reshape(n, ub)
    bad = np.nonzero((a != b).any(axis=1))[0]
    print(f"n={n}: bad units {len(bad)}; statuses {np.unique(ust.cpu().numpy())}; lens {np.unique(ulen.cpu().numpy())}")
    for u in bad[:4]:
        d = np.nonzero(a[u] != b[u])[0]
        lines = sorted(set((d // 128).tolist()))
        print(f"  unit {u}: {len(d)} bytes differ, lines {lines[:12]}{'...' if len(lines) > 12 else ''}; "
              f"0xEE-bytes {(b[u][d] == 0xEE).sum()}; first diff at {d[0]}: got {b[u][d[0]:d[0]+8].tolist()} want {a[u][d[0]:d[0]+8].tolist()}")
