#!/usr/bin/env python3
"""Phase cycles of the one-tile encoders (diagnostic build CPK_EM_PROF, CPK_LIB=lib_exp/em_prof.so):
encode_batch of 1M x 4 KiB units (encode_unit) against encode_message_batch of 1M messages of
4 segments x 127 words (encode_message_one), cycles per unit per wave (s_memtime)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "capnp-zig_amd"))
import torch
import capnp_packed as cp

thr = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n, ub, segs, sw = 1 << 20, 4096, 4, 127
dev = torch.device("cuda", 0)
L = cp.lib()
f = L.capnp_packed_debug_em_prof
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
reps = 3
# plain encode
d_in = cp.generate(n, ub, seed=0xC0DE0003, zero_thresh=thr, device=dev)
in_off, in_len = cp.uniform_layout(n, ub, device=dev)
slot = cp.encode_bound(ub)
pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
plen = torch.zeros(n, dtype=torch.int64, device=dev)
pst = torch.zeros(n, dtype=torch.int32, device=dev)
cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
torch.cuda.synchronize()
f(buf)
for _ in range(reps):
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
torch.cuda.synchronize()
f(buf)
unit = [buf[i] / (reps * n) for i in range(4)]
del d_in
# fused framing encode
sb = 8 * sw
pool = cp.generate(n * segs, sb, seed=0xC0DE0006, zero_thresh=thr, device=dev)
seg_ptr = pool.data_ptr() + torch.arange(n * segs, dtype=torch.int64, device=dev) * sb
seg_len = torch.full((n * segs,), sb, dtype=torch.int64, device=dev)
first = torch.arange(0, n * segs, segs, dtype=torch.int32, device=dev)
count = torch.full((n,), segs, dtype=torch.int32, device=dev)
fb = 8 * 3 + segs * sb
mslot = (cp.encode_bound(fb) + 15) // 16 * 16
m_off, m_cap = cp.uniform_layout(n, mslot, device=dev)
m_cap.fill_(cp.encode_bound(fb))
d_m = torch.empty(n * mslot, dtype=torch.uint8, device=dev)
mlen = torch.zeros(n, dtype=torch.int64, device=dev)
mst = torch.zeros(n, dtype=torch.int32, device=dev)
cp.encode_message_batch(seg_ptr, seg_len, first, count, d_m, m_off, m_cap, mlen, mst)
torch.cuda.synchronize()
f(buf)
for _ in range(reps):
    cp.encode_message_batch(seg_ptr, seg_len, first, count, d_m, m_off, m_cap, mlen, mst)
torch.cuda.synchronize()
f(buf)
msg = [buf[i] / (reps * n) for i in range(4, 8)]
names = ["prologue", "stage", "tile", "total"]
print(json.dumps({"thr": thr, "encode_unit": dict(zip(names, [round(x) for x in unit])),
                  "encode_message_one": dict(zip(names, [round(x) for x in msg])),
                  "ok": bool((pst == 0).all().item() and (mst == 0).all().item())}))
