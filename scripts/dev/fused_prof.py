#!/usr/bin/env python3
"""Phase cycle breakdown of decode_fused_kernel (diagnostic build CPK_LIB=.../lib_exp/prof.so)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "capnp-zig_amd"))
import torch
import capnp_packed as cp

thr = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n, ub = 1 << 20, 4096
dev = torch.device("cuda", 0)
d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=thr, device=dev)
in_off, in_len = cp.uniform_layout(n, ub, device=dev)
slot = cp.encode_bound(ub)
pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
plen = torch.zeros(n, dtype=torch.int64, device=dev)
pst = torch.zeros(n, dtype=torch.int32, device=dev)
cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
ulen = torch.zeros(n, dtype=torch.int64, device=dev)
ust = torch.zeros(n, dtype=torch.int32, device=dev)
L = cp.lib()
f = L.capnp_packed_debug_fill_prof
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
torch.cuda.synchronize()
f(buf)
reps = 3
for _ in range(reps):
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
torch.cuda.synchronize()
f(buf)
names = ["wait", "stage+issue", "map", "fix", "scan+serial", "count", "codewalk", "expand"]
per_unit = {nm: round(buf[i] / (reps * n), 1) for i, nm in enumerate(names)}
per_unit["total"] = round(sum(buf) / (reps * n), 1)
print(json.dumps({"thr": thr, "cycles_per_unit_per_wave": per_unit, "roundtrip": bool(torch.equal(d_out, d_in))}))
