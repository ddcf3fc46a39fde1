#!/usr/bin/env python3
"""Dev: where a warm PackedConnections.handle_read spends its time (4096 connections x 16
messages of 4 KiB): readv_raw (native call + buffers), the per-connection grouping into frame
views, handle_read's result dict, and dropping the previous read's result. FR_BALLAST=N first
creates N million live Python objects (a process holding a large heap, as the full bench does)."""
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
ballast = [[i] for i in range(int(float(os.environ.get("FR_BALLAST", "0")) * 1e6))]
# FR_PRE=dense,read_message,framing,c5: run those bench legs first (the full bench's process state)
if os.environ.get("FR_PRE"):
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    import bench
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    legs = {"dense": bench.dense_leg, "read_message": bench.read_message_leg, "framing": bench.message_leg,
            "c5": bench.skewed_leg, "validate": bench.validate_leg}
    for name in os.environ["FR_PRE"].split(","):
        t = time.perf_counter()
        legs[name](args, dev)
        torch.cuda.empty_cache()
        print(f"pre-leg {name} {time.perf_counter() - t:.1f} s", flush=True)
    if os.environ.get("FR_RELEASE"):  # drop the side streams the legs' batches created
        rc = cp.lib().capnp_packed_stream_release(torch.cuda.current_stream().cuda_stream)
        print(f"stream_release rc={rc}", flush=True)
print(f"ballast {len(ballast)} objects", flush=True)
T = {}
sess_cls = cp.FramerSession
orig_raw, orig_read = sess_cls.readv_raw, sess_cls._read


def raw(self, reads):
    t = time.perf_counter()
    r = orig_raw(self, reads)
    T["readv_raw"] = T.get("readv_raw", 0) + time.perf_counter() - t
    return r


def rd(self, reads):
    t = time.perf_counter()
    r = orig_read(self, reads)
    T["_read"] = T.get("_read", 0) + time.perf_counter() - t
    return r


sess_cls.readv_raw, sess_cls._read = raw, rd
pc = cp.PackedConnections(conns, device=dev)
res = None
for r in range(5):
    T.clear()
    t0 = time.perf_counter()
    new = pc.handle_read(streams)
    t1 = time.perf_counter()
    res = new
    t2 = time.perf_counter()
    if os.environ.get("FR_VERIFY"):  # the bench leg's check between reads: CPU reads of a few frames
        for c in (0, conns // 2, conns - 1):
            assert all(len(bytes(x)) == 4096 for x in res[c])
    print(f"read {r}: handle_read {1e3 * (t1 - t0):.2f} ms (readv_raw {1e3 * T['readv_raw']:.2f}, grouping "
          f"{1e3 * (T['_read'] - T['readv_raw']):.2f}, result {1e3 * (t1 - t0 - T['_read']):.2f}), "
          f"drop previous {1e3 * (t2 - t1):.2f} ms", flush=True)
