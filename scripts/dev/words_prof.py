#!/usr/bin/env python3
"""Phase cycles of decode_words_kernel per wave (dev build with -DCPK_FILL_PROF=1, selected with
CPK_LIB=capnp-zig_amd/lib_exp/words_prof.so). s_memtime ticks summed over each wave's rounds:
wait (ring loads), ring (shift + writes + next loads), steps, stores, total; plus steps and
sub-rounds per wave. Usage: CPK_LIB=... python3 scripts/dev/words_prof.py [thr ...]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "capnp-zig_amd"))
import torch  # noqa: E402

import capnp_packed as cp  # noqa: E402

n, ub = 1 << 20, 4096
dev = torch.device("cuda", 0)
L = cp.lib()
f = L.capnp_packed_debug_fill_prof
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
for thr in [int(x) for x in (sys.argv[1:] or ["128", "26", "230"])]:
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
    buf = (ctypes.c_ulonglong * 8)()
    with cp.decoder("words"):
        cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
        torch.cuda.synchronize()
        f(buf)
        reps = 3
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(reps):
            cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, in_len, ulen, ust)
        ev1.record()
        torch.cuda.synchronize()
        f(buf)
    waves = reps * n // 64
    names = ["wait_loads", "ring", "chain", "words", "flush", "steps_n", "subrounds_n", "total"]
    out = {nm: round(buf[i] / waves, 1) for i, nm in enumerate(names)}
    print(json.dumps({"thr": thr, "ms": round(ev0.elapsed_time(ev1) / reps, 4), "per_wave": out,
                      "roundtrip": bool(torch.equal(d_out, d_in))}), flush=True)
    del d_in, d_pk, d_out
    torch.cuda.empty_cache()
