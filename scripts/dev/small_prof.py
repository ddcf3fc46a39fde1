#!/usr/bin/env python3
"""Dev: small-unit decode alone (C5's size law clipped to the small class), decode time
with HIP events; with CPK_LIB=.../lib_exp/prof.so also the group kernel's phase cycles."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "capnp-zig_amd"))
import numpy as np
import torch
import capnp_packed as cp

n = 1 << 20
u = np.random.default_rng(0xC0DE0005).random(n)
sizes = (8 * np.floor(np.clip(64.0 * (1.0 - u) ** (-1.0 / 1.1), 64, 640) / 8)).astype(np.int64)
dev = torch.device("cuda", 0)
sz = torch.from_numpy(sizes).to(dev)
in_off = torch.zeros(n, dtype=torch.int64, device=dev)
in_off[1:] = torch.cumsum(sz, 0)[:-1]
U = int(sizes.sum())
d_in = cp.generate(1, U, seed=0xC0DE0005, zero_thresh=int(sys.argv[1]) if len(sys.argv) > 1 else 128, device=dev)
caps = (sz // 8) * 10
slots = (caps + 15) // 16 * 16
pk_off = torch.zeros(n, dtype=torch.int64, device=dev)
pk_off[1:] = torch.cumsum(slots, 0)[:-1]
d_pk = torch.empty(int(slots.sum().item()), dtype=torch.uint8, device=dev)
plen = torch.zeros(n, dtype=torch.int64, device=dev)
pst = torch.zeros(n, dtype=torch.int32, device=dev)
cp.encode_batch(d_in, in_off, sz, d_pk, pk_off, caps, plen, pst)
d_out = torch.empty(U, dtype=torch.uint8, device=dev)
ulen = torch.zeros(n, dtype=torch.int64, device=dev)
ust = torch.zeros(n, dtype=torch.int32, device=dev)
dec = lambda: cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, sz, ulen, ust)  # noqa: E731
dec()
torch.cuda.synchronize()
L = cp.lib()
prof = hasattr(L, "capnp_packed_debug_fill_prof")
buf = (ctypes.c_ulonglong * 8)()
if prof:
    L.capnp_packed_debug_fill_prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    L.capnp_packed_debug_fill_prof(buf)
reps = 5
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    dec()
e1.record()
torch.cuda.synchronize()
ok = bool(torch.equal(d_out, d_in) and (ust == 0).all().item())
res = {"small": os.environ.get("CPK_SMALL", "group"), "units": n, "U": U, "P": int(plen.sum().item()),
       "decode_ms": round(e0.elapsed_time(e1) / reps, 4), "ok": ok}
if prof:
    L.capnp_packed_debug_fill_prof(buf)
    groups = buf[5] or 1
    res["cycles_per_group"] = {k: round(buf[i] / groups, 1) for i, k in enumerate(["meta", "load", "decode", "store"])}
    res["units_per_group"] = round(buf[4] / groups, 1)
print(json.dumps(res))
