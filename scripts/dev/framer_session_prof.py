#!/usr/bin/env python3
"""Dev: where the rpc_framer leg's time goes on the framer session: FramerSession.read (native
rounds + Python frame views) against PackedConnections.handle_read, warm session, and the native
call's round count (4096 connections x 16 messages of 4 KiB)."""
import os, struct, sys, time
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
sess = cp.FramerSession(conns)
for r in range(int(os.environ.get("FR_REPS", "4"))):
    t0 = time.perf_counter()
    fr, st = sess.read(streams)
    t1 = time.perf_counter()
    print(f"session.read {1e3 * (t1 - t0):.2f} ms, frames {sum(len(v) for v in fr.values())}", flush=True)
pc = cp.PackedConnections(conns, device=dev)
for r in range(int(os.environ.get("FR_REPS", "4"))):
    t0 = time.perf_counter()
    res = pc.handle_read(streams)
    t1 = time.perf_counter()
    print(f"handle_read {1e3 * (t1 - t0):.2f} ms", flush=True)
# the host-side input assembly alone (what read() does before the native call)
t0 = time.perf_counter()
lens = np.zeros(conns, dtype=np.uint64)
for c, d in streams.items():
    lens[c] = len(d)
host = np.empty(int(lens.sum()), dtype=np.uint8)
o = np.zeros(conns, dtype=np.uint64)
o[1:] = np.cumsum(lens)[:-1]
for c, d in streams.items():
    host[int(o[c]):int(o[c]) + len(d)] = np.frombuffer(d, dtype=np.uint8)
print(f"host assembly {1e3 * (time.perf_counter() - t0):.2f} ms")
# the native call's share of a warm session read
L = cp.lib()
native = L.capnp_packed_framer_read
acc = []


def timed(*a):
    t = time.perf_counter()
    r = native(*a)
    acc.append(time.perf_counter() - t)
    return r


L.capnp_packed_framer_read = timed
for r in range(3):
    acc.clear()
    t0 = time.perf_counter()
    fr, st = sess.read(streams)
    t1 = time.perf_counter()
    print(f"session.read {1e3 * (t1 - t0):.2f} ms: native {1e3 * sum(acc):.2f} ms in {len(acc)} call(s)", flush=True)
L.capnp_packed_framer_read = native
