#!/usr/bin/env python3
"""Single-buffer crossover for the Zig drop-in: latency of one
packPacked / unpackPacked call through the C-ABI single-buffer entry points
(capnp_packed_encode / capnp_packed_decode: H2D, kernels, D2H, sync) against the CPU
oracle on one core (oracle/packed_oracle.c, a restatement of message.zig:88-271), for one
unit of 64 B .. 16 MiB of the bench's byte distribution at p = 0.1, 0.5 and 0.9 (zero-byte
thresholds 26 / 128 / 230, or those given on the command line). GPU unpack goes through the
Zig binding's path (zig/packed_ffi.zig unpackPacked): one capnp_packed_decode into a buffer
of max(4096, 4 x packed), retried once at the size an OUT_OF_SPACE reports (zero-heavy
units expand past 4x). Prints one JSON object; per density, the threshold is the smallest
size from which the GPU call is faster."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "capnp-zig_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

import capnp_packed as cp  # noqa: E402
import oracle  # noqa: E402


def t_us(fn, budget=0.3, max_reps=2000):
    fn()
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or (time.perf_counter() - t0 < budget and reps < max_reps):
        fn()
        reps += 1
    return (time.perf_counter() - t0) / reps * 1e6


def density(thr):
    import ctypes
    L, O = cp.lib(), oracle.lib()
    rows = []
    size = 64
    while size <= 16 << 20:
        data = oracle.generate(1, size, seed=0xC0DE0008, zero_thresh=thr).tobytes()
        st, packed = oracle.pack(data)
        assert st == 0
        assert cp.pack_packed(data) == packed and cp.unpack_packed(packed) == data
        # caller-owned buffers, allocated once: the timings are the calls a Zig caller makes
        # (the output allocation is the same on both sides and left out)
        src_u = ctypes.create_string_buffer(data, max(1, len(data)))
        src_p = ctypes.create_string_buffer(packed, max(1, len(packed)))
        cap_p = 10 * (size // 8) + 16
        dst_p = ctypes.create_string_buffer(cap_p)
        guess = max(4096, 4 * len(packed))  # packed_ffi.zig unpackPacked's first capacity
        dst_u = ctypes.create_string_buffer(max(guess, size))
        n = ctypes.c_size_t()

        def cpu_pack():
            O.oracle_pack(src_u, size, dst_p, cap_p, ctypes.byref(n))

        def cpu_unpack():  # unpackPacked: estimateUnpackedSize, then the decode
            O.oracle_estimate_unpacked_size(src_p, len(packed), ctypes.byref(n))
            O.oracle_unpack(src_p, len(packed), dst_u, n.value, ctypes.byref(n))

        def cpu_size():
            O.oracle_estimate_unpacked_size(src_p, len(packed), ctypes.byref(n))

        def gpu_pack():
            assert L.capnp_packed_encode(src_u, size, dst_p, cap_p, ctypes.byref(n)) == 0

        def gpu_unpack():  # the binding's calls: a 4x guess, one retry at the reported size
            st = L.capnp_packed_decode(src_p, len(packed), dst_u, guess, ctypes.byref(n))
            if st == cp.OUT_OF_SPACE and n.value > guess:
                st = L.capnp_packed_decode(src_p, len(packed), dst_u, n.value, ctypes.byref(n))
            assert st == 0

        def gpu_size():
            assert L.capnp_packed_decoded_size(src_p, len(packed), ctypes.byref(n)) == 0

        row = {"bytes": size, "packed": len(packed), "retry": 4 * len(packed) < size and size > 4096,
               "cpu_pack_us": t_us(cpu_pack), "cpu_unpack_us": t_us(cpu_unpack),
               "gpu_pack_us": t_us(gpu_pack), "gpu_unpack_us": t_us(gpu_unpack),
               "cpu_size_us": t_us(cpu_size), "gpu_size_us": t_us(gpu_size)}
        assert dst_u.raw[:size] == data
        rows.append({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
        size *= 4
    out = {"zero_thresh": thr, "rows": rows}
    for op in ("pack", "unpack", "size"):
        win = [r["bytes"] for r in rows if r[f"gpu_{op}_us"] < r[f"cpu_{op}_us"]]
        out[f"{op}_gpu_faster_from_bytes"] = min(win) if win else None
    return out


def main():
    thrs = [int(a) for a in sys.argv[1:]] or [26, 128, 230]
    out = {"densities": [density(t) for t in thrs]}
    out["note"] = ("one unit per call through the C entry points with caller-owned buffers allocated "
                   "once; GPU = single-buffer C-ABI (pageable caller buffers staged through pinned memory, "
                   "one H2D + launches + D2H + sync; unpack = capnp_packed_decode at the Zig binding's 4x guess, "
                   "retried once at the reported size when it does not fit, "
                   "size = capnp_packed_decoded_size); CPU = oracle/packed_oracle.c, one thread "
                   "(unpack = size pass + decode, as message.zig:88-145)")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
