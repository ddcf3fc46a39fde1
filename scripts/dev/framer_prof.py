#!/usr/bin/env python3
"""Dev: phase timings of PackedConnections.handle_read on the bench's framer workload."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np
import torch
import bench
import capnp_packed as cp

class A: zero_thresh = 128
dev = torch.device("cuda", 0)
conns, msgs = 4096, 16
n = conns * msgs
d_fr = cp.generate(n, 4096, seed=0xC0DE0007, zero_thresh=128, device=dev)
import struct
d_fr.view(n, 4096)[:, :8] = torch.tensor(list(struct.pack("<II", 0, 511)), dtype=torch.uint8, device=dev)
off, ln = cp.uniform_layout(n, 4096, device=dev)
slot = cp.encode_bound(4096)
pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
d_pk = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
plen = torch.zeros(n, dtype=torch.int64, device=dev); pst = torch.zeros(n, dtype=torch.int32, device=dev)
cp.encode_batch(d_fr, off, ln, d_pk, pk_off, pk_cap, plen, pst); torch.cuda.synchronize()
pk_h, pl_h = d_pk.cpu().numpy(), plen.cpu().numpy()
streams = {c: b"".join(pk_h[i * slot:i * slot + int(pl_h[i])].tobytes() for i in range(c * msgs, (c + 1) * msgs))
           for c in range(conns)}
total = sum(len(v) for v in streams.values())
for rep in range(3):
    pc = cp.PackedConnections(conns)
    t = [time.perf_counter()]
    for c, data in streams.items(): pc.framers[c].push(data)
    t.append(time.perf_counter())
    host = np.frombuffer(b"".join(bytes(pc.framers[c].buffer) for c in range(conns)), dtype=np.uint8)
    t.append(time.perf_counter())
    lens = np.array([len(streams[c]) for c in range(conns)], dtype=np.uint64)
    base = np.zeros(conns, dtype=np.uint64); base[1:] = np.cumsum(lens)[:-1]
    guess = np.full(conns, 8192, dtype=np.uint64)
    frames_cap = 8 * total + 8 * int(guess.sum())
    frames = np.empty(frames_cap, dtype=np.uint8)
    mf = total // 2 + conns + 1
    f_off = np.empty(mf, dtype=np.uint64); f_len = np.empty(mf, dtype=np.uint64); f_conn = np.empty(mf, dtype=np.uint32)
    consumed = np.zeros(conns, dtype=np.uint64); status = np.zeros(conns, dtype=np.int32); nf = ctypes.c_uint32(0)
    t.append(time.perf_counter())
    st = cp.lib().capnp_packed_frame_connections(host.ctypes.data, total, base.ctypes.data, lens.ctypes.data, conns,
        guess.ctypes.data, frames.ctypes.data, frames_cap, f_off.ctypes.data, f_len.ctypes.data, f_conn.ctypes.data,
        mf, consumed.ctypes.data, status.ctypes.data, ctypes.byref(nf))
    t.append(time.perf_counter())
    pc2 = cp.PackedConnections(conns)
    t2 = time.perf_counter(); res = pc2.handle_read(streams); t3 = time.perf_counter()
    d = np.diff(t) * 1e3
    print(f"st={st} nf={nf.value} push {d[0]:.1f} join {d[1]:.1f} alloc {d[2]:.1f} native {d[3]:.1f} ms | handle_read {1e3*(t3-t2):.1f} ms")
