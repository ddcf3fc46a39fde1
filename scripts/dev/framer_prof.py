#!/usr/bin/env python3
"""Dev: where capnp_packed_frame_connections' time goes (bench rpc_framer's workload): the
native call alone with pageable / pinned input and frames, and PackedConnections.handle_read."""
import ctypes, os, struct, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "capnp-zig_amd"))
import numpy as np
import torch
import capnp_packed as cp

dev = torch.device("cuda", 0)
conns, msgs = 4096, 16
n = conns * msgs
d_fr = cp.generate(n, 4096, seed=0xC0DE0007, zero_thresh=128, device=dev)
d_fr.view(n, 4096)[:, :8] = torch.tensor(list(struct.pack("<II", 0, 511)), dtype=torch.uint8, device=dev)
off, ln = cp.uniform_layout(n, 4096, device=dev)
slot = cp.encode_bound(4096)
pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
d_pk = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
plen = torch.zeros(n, dtype=torch.int64, device=dev)
pst = torch.zeros(n, dtype=torch.int32, device=dev)
cp.encode_batch(d_fr, off, ln, d_pk, pk_off, pk_cap, plen, pst)
torch.cuda.synchronize()
pk_h, pl_h = d_pk.cpu().numpy(), plen.cpu().numpy()
streams = {c: b"".join(pk_h[i * slot:i * slot + int(pl_h[i])].tobytes() for i in range(c * msgs, (c + 1) * msgs))
           for c in range(conns)}
lens = np.array([len(streams[c]) for c in range(conns)], dtype=np.uint64)
base = np.zeros(conns, dtype=np.uint64)
base[1:] = np.cumsum(lens)[:-1]
total = int(lens.sum())
joined = np.frombuffer(b"".join(streams[c] for c in range(conns)), dtype=np.uint8)
frames_cap = 4 * total + 2 * 8192 * conns
max_frames = total // 64 + conns + 16
L = cp.lib()

import mmap
keep = []
def alloc_out(kind):
    if kind == "pin":
        return torch.empty(frames_cap, dtype=torch.uint8, pin_memory=True).numpy()
    if kind == "huge":  # anonymous mapping advised for transparent huge pages
        mm = mmap.mmap(-1, frames_cap, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        mm.madvise(mmap.MADV_HUGEPAGE)
        return np.frombuffer(mm, dtype=np.uint8)
    return np.empty(frames_cap, dtype=np.uint8)

def native(pinned_in, pinned_out, reps=3, fresh=None):
    best = 1e9
    hin = torch.empty(total, dtype=torch.uint8, pin_memory=True).numpy() if pinned_in else np.empty(total, dtype=np.uint8)
    hin[:] = joined
    fr = torch.empty(frames_cap, dtype=torch.uint8, pin_memory=True).numpy() if pinned_out else np.empty(frames_cap, dtype=np.uint8)
    for _ in range(reps):
        if fresh:
            fr = alloc_out(fresh)
            keep.append(fr)  # held, as a caller holds its frames
        g = np.full(conns, 8192, dtype=np.uint64)
        f_off = np.empty(max_frames, dtype=np.uint64); f_len = np.empty(max_frames, dtype=np.uint64)
        f_conn = np.empty(max_frames, dtype=np.uint32)
        cons = np.zeros(conns, dtype=np.uint64); st = np.zeros(conns, dtype=np.int32); nf = ctypes.c_uint32(0)
        t0 = time.perf_counter()
        r = L.capnp_packed_frame_connections(hin.ctypes.data, total, base.ctypes.data, lens.ctypes.data, conns,
                                             g.ctypes.data, fr.ctypes.data, frames_cap, f_off.ctypes.data,
                                             f_len.ctypes.data, f_conn.ctypes.data, max_frames, cons.ctypes.data,
                                             st.ctypes.data, ctypes.byref(nf))
        best = min(best, time.perf_counter() - t0)
        assert r == 0 and nf.value == n, (r, nf.value)
    return round(best * 1e3, 2)

out = {}
try:
    out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
except OSError:
    out["thp"] = "?"
for fk in ("page", "huge"):
    out[f"native fresh out={fk} ms"] = native(False, False, fresh=fk)
keep.clear()
for pi in (False, True):
    for po in (False, True):
        out[f"native in={'pin' if pi else 'page'} out={'pin' if po else 'page'} ms"] = native(pi, po)
t0 = time.perf_counter(); a = torch.empty(frames_cap, dtype=torch.uint8, pin_memory=True); out["pin_alloc_first_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
del a
t0 = time.perf_counter(); a = torch.empty(frames_cap, dtype=torch.uint8, pin_memory=True); out["pin_alloc_cached_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
del a
import cProfile, pstats, io
for rep in range(3):
    pc = cp.PackedConnections(conns, device=dev)
    t0 = time.perf_counter(); res = pc.handle_read(streams); out[f"handle_read_{rep}_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
print(out)
pc = cp.PackedConnections(conns, device=dev)
pr = cProfile.Profile(); pr.enable(); res = pc.handle_read(streams); pr.disable()
sio = io.StringIO(); pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(12); print(sio.getvalue()[:3000])
# Python phases of handle_read (its input layout and the frames' memoryviews), replicated
t0 = time.perf_counter()
host = np.empty(total, dtype=np.uint8)
for c in range(conns):
    b = int(base[c]); host[b:b + int(lens[c])] = np.frombuffer(streams[c], dtype=np.uint8)
t1 = time.perf_counter()
fr = np.empty(frames_cap, dtype=np.uint8)
view = memoryview(fr).toreadonly()
offs = list(range(0, n * 4096, 4096))
lst = [view[o:o + 4096] for o in offs]
t2 = time.perf_counter()
import gc
gc.disable(); lst2 = [view[o:o + 4096] for o in offs]; gc.enable()
t3 = time.perf_counter()
print({"memoryviews_nogc_ms": round((t3 - t2) * 1e3, 2)})
print({"layout_ms": round((t1 - t0) * 1e3, 2), "memoryviews_ms": round((t2 - t1) * 1e3, 2)})
