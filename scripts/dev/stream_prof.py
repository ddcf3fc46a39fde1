#!/usr/bin/env python3
"""Phase breakdown of decode_stream_kernel (diagnostic build: CPK_LIB=capnp-zig_amd/lib_exp/stream_prof.so)."""
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
f = cp.lib().capnp_packed_debug_stream_prof
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
torch.cuda.synchronize()
f(buf)
reps = 3
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(reps):
    cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
ev[1].record()
torch.cuda.synchronize()
f(buf)
waves = reps * n // 64
names = ["round_start", "-", "flush", "iterations", "flushes", "rounds", "total"]
out = {nm: round(buf[i] / waves, 1) for i, nm in enumerate(names) if nm != "-"}
out["cycles_per_iteration"] = round((buf[6] - buf[0] - buf[2]) / max(1, buf[3]), 1)
print(json.dumps({"thr": thr, "per_wave": out, "ms": ev[0].elapsed_time(ev[1]) / reps,
                  "roundtrip": bool(torch.equal(d_out, d_in))}))
