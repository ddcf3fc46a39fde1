#!/usr/bin/env python3
"""Benchmark: device-resident packed encode+decode of independent units.

BASELINE.json metric: "GiB/s device-resident packed encode+decode, 1M x 4KiB
segments, 1/2/4/8 GPU". One step = one batch pass of the hot path:
  encode (packPacked, message.zig:200-271) of every unit into capacity slots,
  decode (unpackPacked, message.zig:88-145) straight from those slots,
  per-rank packed total + RCCL all-gather of the per-rank totals (N > 1).
value = sum over ranks of unpacked bytes per step / max-over-ranks step time, in GiB/s.

Inputs are generated on device before timing (synthetic, counter-based hash:
DESIGN.md §4). After timing, decode(encode(x)) == x is checked on device.

The headline config is BASELINE config 3 (1M x 4 KiB, zero-byte density sweep
10/50/90 %): `value` is the p = 0.5 step; `sweep` times every density, each with
its own encode/decode roofline fraction.

Run: python bench.py [--gpus N --steps K --warmup W]
     --gpus N without a torchrun environment: this process starts N ranks (one per
     GPU, RCCL) as child processes before anything touches a GPU, and exits with
     their status; under torchrun (WORLD_SIZE set) each process is one rank.
     --dry-run: the same launcher on the CPU (gloo), each rank packing a small shard
     with the oracle: checks the rank plumbing and the all-gather without a GPU.
     --same-gpu: a rehearsal of the N-rank GPU step on a one-GPU box: every rank on
     cuda:0 and gloo collectives over host copies (RCCL needs a GPU per rank). The
     ranks share the card, so its `value` is not a scaling number.
"""
import argparse
import json
import statistics
import socket
import struct
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "capnp-zig_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import capnp_packed as cp  # noqa: E402
import sharding  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, 8.0 TB/s (MI355X_MICROARCH.md, chip table)
META_BYTES_PER_UNIT = 44  # in_off, in_len, out_off, out_cap (4 x 8 B read) + out_len (8 B) + status (4 B)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--units", type=int, default=1 << 20, help="units per GPU")
    ap.add_argument("--unit-bytes", type=int, default=4096)
    ap.add_argument("--zero-thresh", type=int, default=128, help="zero-byte probability x 256 (128 = 0.5)")
    ap.add_argument("--seed", type=int, default=0xC0DE0003)
    ap.add_argument("--no-sweep", action="store_true", help="skip the p = 0.1 / 0.9 legs of the density sweep")
    ap.add_argument("--sweep", action="store_true", help=argparse.SUPPRESS)  # the sweep is the default now
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="wall budget of each CPU baseline leg")
    ap.add_argument("--no-dense", action="store_true", help="skip the dense packed-stream decode leg")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 bench-message leg")
    ap.add_argument("--dry-run", action="store_true", help="CPU (gloo) rehearsal of the multi-rank path")
    ap.add_argument("--same-gpu", action="store_true",
                    help="rehearsal on one GPU: all ranks on cuda:0, gloo collectives (not a scaling number)")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-memory leg")
    ap.add_argument("--no-read-message", action="store_true", help="skip the Reader.readPackedMessage leg")
    ap.add_argument("--no-skewed", action="store_true", help="skip the skewed-size config C5 leg")
    ap.add_argument("--no-validate", action="store_true", help="skip the Message.validate leg")
    ap.add_argument("--no-ceilings", action="store_true", help="skip the HBM ceiling sweep (headline-only traces)")
    ap.add_argument("--only", default="", help=argparse.SUPPRESS)  # dev: run one side leg (validate, c5, ...)
    ap.add_argument("--decoder", default="", help=argparse.SUPPRESS)  # dev: capnp_packed_set_decoder name
    return ap.parse_args()


class Workload:
    def __init__(self, n, ub, seed, thr, unit_base, dev):
        self.n, self.ub = n, ub
        self.d_in = cp.generate(n, ub, seed=seed, zero_thresh=thr, unit_base=unit_base, device=dev)
        self.in_off, self.in_len = cp.uniform_layout(n, ub, device=dev)
        self.slot = cp.encode_bound(ub)
        self.pk_off, self.pk_cap = cp.uniform_layout(n, self.slot, device=dev)
        self.d_pk = torch.empty(n * self.slot, dtype=torch.uint8, device=dev)
        self.plen = torch.zeros(n, dtype=torch.int64, device=dev)
        self.pst = torch.zeros(n, dtype=torch.int32, device=dev)
        self.d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
        self.ulen = torch.zeros(n, dtype=torch.int64, device=dev)
        self.ust = torch.zeros(n, dtype=torch.int32, device=dev)

    def encode(self, stream):
        cp.encode_batch(self.d_in, self.in_off, self.in_len, self.d_pk, self.pk_off, self.pk_cap,
                        self.plen, self.pst, stream=stream)

    def decode(self, stream):
        cp.decode_batch(self.d_pk, self.pk_off, self.plen, self.d_out, self.in_off, self.in_len,
                        self.ulen, self.ust, stream=stream)

    def verify(self):
        ok = bool((self.pst == 0).all().item() and (self.ust == 0).all().item()
                  and (self.ulen == self.ub).all().item() and torch.equal(self.d_out, self.d_in))
        return ok


def _host_collectives():
    return dist.is_initialized() and dist.get_backend() == "gloo"


def time_steps(wl, steps, warmup, world, dev):
    stream = torch.cuda.current_stream()
    gathered = [torch.zeros(world, dtype=torch.int64, device=dev)]

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        wl.encode(stream)
        if ev is not None:
            ev[1].record(stream)
        wl.decode(stream)
        if ev is not None:
            ev[2].record(stream)
        # per-rank packed total -> RCCL all-gather (the only collective);
        # gloo (the --same-gpu rehearsal) gathers a host copy
        total = wl.plen.sum()
        gathered[0] = sharding.gather_packed_totals(total.cpu() if _host_collectives() else total)

    for _ in range(warmup):
        step()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in events) / steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in events) / steps
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device="cpu" if _host_collectives() else dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    return float(elapsed.item()), enc_ms, dec_ms, gathered[0]


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_native():
    """The oracle (tests/oracle.py) bound to a -O3 -march=native build of
    oracle/packed_oracle.c made for THIS host (falls back to the prebuilt
    x86-64-v2 liboracle.so if gcc fails). Returns (module, march)."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import tempfile
    import oracle
    srcs = [os.path.join(HERE, "oracle", f) for f in ("packed_oracle.c", "packed_fast.c")]
    out = os.path.join(tempfile.gettempdir(), f"cpk_oracle_native_{os.getpid()}.so")
    try:
        subprocess.run(["gcc", "-O3", "-march=native", "-fPIC", "-fopenmp", "-std=c11", "-shared", "-o", out] + srcs,
                       check=True, capture_output=True, timeout=120)
        oracle._lib, oracle.LIB_PATH = None, out
        oracle.lib()
        return oracle, "native"
    except Exception:
        oracle._lib, oracle.LIB_PATH = None, os.path.join(HERE, "oracle", "liboracle.so")
        return oracle, "x86-64-v2"


def _cpu_leg(oracle, args, n, threads, budget_s, fast=True):
    """pack + unpack of n units, repeated until budget_s is spent: the word-at-a-time port
    (oracle/packed_fast.c, fast=True) or the checker itself."""
    import numpy as np
    pack = oracle.fast_pack_batch if fast else oracle.pack_batch
    unpack = oracle.fast_unpack_batch if fast else oracle.unpack_batch
    ub = args.unit_bytes
    data = oracle.generate(n, ub, seed=args.seed, zero_thresh=args.zero_thresh, threads=threads)
    in_off = np.arange(0, n * ub + 1, ub, dtype=np.uint64)
    slot = 10 * ub // 8
    pk_off = np.arange(0, n * slot + 1, slot, dtype=np.uint64)
    out, out_len, st = pack(data, in_off, pk_off, threads=threads)
    dense_off = np.zeros(n + 1, dtype=np.uint64)
    dense_off[1:] = np.cumsum(out_len)
    dense = np.concatenate([out[int(pk_off[i]):int(pk_off[i]) + int(out_len[i])] for i in range(n)])
    # output buffers allocated and written once before the timed region and reused, as the GPU
    # leg's are: fresh np.zeros pages fault in inside the call, and the page faults of many
    # threads serialise in the kernel (the all-core leg scaled ~3x over 16 threads with them)
    pbufs = (out, out_len, st)
    ubufs = unpack(dense, dense_off, in_off, threads=threads)
    reps, t_total = 0, 0.0
    while t_total < budget_s and reps < 1000:
        t0 = time.perf_counter()
        out, out_len, st = pack(data, in_off, pk_off, threads=threads, bufs=pbufs)
        dec, dec_len, dst = unpack(dense, dense_off, in_off, threads=threads, bufs=ubufs)
        t_total += time.perf_counter() - t0
        reps += 1
    assert (st == 0).all() and (dst == 0).all() and (dec[:n * ub] == data).all()
    return reps * n * ub / t_total / 2 ** 30, reps, t_total


def cpu_baseline(args, budget_s):
    """The codec on this host's cores, same generator and unit size/density as the GPU,
    OpenMP over units, bounded samples: an all-core leg on 32K units (128 MiB, past the LLC)
    and a 1-core leg on 2K units. `value` is the word-at-a-time port (oracle/packed_fast.c:
    message.zig:88-271's algorithm and record choices, SWAR masks, BMI2 pext / pdep, memcpy
    runs; bit-exact against the checker, tests/test_fast_cpu.py), the closest this image gets
    to a ReleaseFast build of the Zig reference (no Zig toolchain here). The checker's own
    1-core rate (oracle/packed_oracle.c, byte by byte) is reported beside it."""
    oracle, march = _oracle_native()
    # the host's CPU share: OMP_NUM_THREADS where the launcher sets it (the GPU box
    # exports 16 per GPU while the affinity mask shows every core), else the affinity
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    allc, reps_a, t_a = _cpu_leg(oracle, args, 32768, cores, budget_s)
    one, reps_1, t_1 = _cpu_leg(oracle, args, 2048, 1, budget_s / 2)
    chk, reps_c, t_c = _cpu_leg(oracle, args, 2048, 1, budget_s / 3, fast=False)
    return {"value": round(allc, 4), "unit": "GiB/s", "cores": cores, "kind": "port",
            "one_core_GiB_s": round(one, 4), "checker_one_core_GiB_s": round(chk, 4),
            "nproc": os.cpu_count(), "cpu_model": _cpu_model(),
            "build": f"gcc -O3 -march={march} -fopenmp",
            "sample": f"pack+unpack of units x {args.unit_bytes} B (same generator/seed/density as the GPU) via "
                      f"oracle/packed_fast.c: all-core {reps_a} x 32768 units in {t_a:.1f} s ({cores} threads), "
                      f"1-core {reps_1} x 2048 units in {t_1:.1f} s; checker (oracle/packed_oracle.c) 1-core "
                      f"{reps_c} x 2048 units in {t_c:.1f} s",
            "note": "word-at-a-time C port of message.zig:88-271 (the reference's records and its size pass "
                    "before the expansion; SWAR, BMI2 pext/pdep, memcpy/memset runs), bit-exact vs the "
                    "checker; the Zig reference itself cannot be built here (no Zig toolchain)"}


def c1_leg(reps_cpu=300, reps_gpu=100):
    """BASELINE config 1: the reference bench's own message (bench/packed_unpacked.zig
    buildMessage, default --payload 4096 --list-len 2048: U = 20,536 B framed,
    P = 18,463 B packed; tests/pyref.py bench_message_segments), pack / unpack /
    roundtrip ns/iter in the bench's byte accounting (:350-357): pack U, unpack P,
    roundtrip U + P. CPU: the oracle, one thread (the bench is single-threaded),
    toPackedBytes = pack(toBytes) and initPacked = unpack + Message.init. GPU: the
    single-buffer C-ABI (capnp_packed_encode / _decode: one unit, H2D + kernels +
    D2H + sync per call). Next to bench/baselines.json:69-183 (Debug build,
    hardware not recorded)."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import oracle
    import pyref
    framed = pyref.frame(pyref.bench_message_segments())
    st, packed = oracle.pack(framed)
    assert st == 0 and len(framed) == 20536 and len(packed) == 18463
    U, P = len(framed), len(packed)

    def t_ns(fn, reps):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps * 1e9

    def cpu_unpack():
        s2, out = oracle.unpack(packed)
        assert s2 == 0 and oracle.message_init(out, 1)[0] == 0

    cpu = {"pack_ns": t_ns(lambda: oracle.pack(framed), reps_cpu), "unpack_ns": t_ns(cpu_unpack, reps_cpu)}
    cpu["roundtrip_ns"] = cpu["pack_ns"] + cpu["unpack_ns"]
    assert cp.pack_packed(framed) == packed and cp.unpack_packed(packed) == framed
    gpu = {"pack_ns": t_ns(lambda: cp.pack_packed(framed), reps_gpu),
           "unpack_ns": t_ns(lambda: cp.Message.init_packed(packed), reps_gpu)}
    gpu["roundtrip_ns"] = gpu["pack_ns"] + gpu["unpack_ns"]
    ref = {"pack_ns": 173923.65, "unpack_ns": 108204.37, "roundtrip_ns": 270675.97}
    acct = {"pack": U, "unpack": P, "roundtrip": U + P}
    out = {"unpacked_len": U, "packed_len": P}
    for name, d in (("cpu_oracle_1core", cpu), ("gpu_single_buffer", gpu), ("reference_debug_ci", ref)):
        out[name] = {k: round(v, 1) for k, v in d.items()}
        out[name].update({f"{m}_MiB_s": round(acct[m] / (d[m + "_ns"] * 1e-9) / 2 ** 20, 1) for m in acct})
    out["note"] = ("ns/iter and MiB/s in the reference bench's accounting (pack U, unpack P, roundtrip U+P); "
                   "reference_debug_ci = bench/baselines.json:69-183 (Debug build, hardware not recorded)")
    return out


def copy_ceiling(dev, nbytes, reps=5):
    """Device-copy ceiling: a torch copy of nbytes (read + write), GB/s (the round-1..4 figure)."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    ev[0].record(stream)
    for _ in range(reps):
        b.copy_(a)
    ev[1].record(stream)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    del a, b
    return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)


def ceilings(dev, nbytes, reps=5):
    """HBM ceilings on this box (verdict r4 item 1a), GB/s, from capnp-zig_amd/lib/libcpk_ceiling.so
    (csrc/bench_ceiling.hip: 16 B per lane, UNR loads in flight, persistent grids, non-temporal):
    the best tuned copy, read-only and write-only streams over a small grid x UNR sweep, and a
    decode-shaped stream (reads 5, writes 8 4-KiB slabs per step: the p = 0.5 decode's P : U).
    `torch_copy` is the plain torch copy the bench reported until round 4."""
    import ctypes
    L = ctypes.CDLL(os.path.join(HERE, "capnp-zig_amd", "lib", "libcpk_ceiling.so"))
    L.cpk_ceiling_stream.restype = ctypes.c_float
    L.cpk_ceiling_stream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    L.cpk_ceiling_shaped.restype = ctypes.c_float
    L.cpk_ceiling_shaped.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    s = torch.cuda.current_stream().cuda_stream
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(1)
    out, cfg = {}, {}
    for kind, name, mult in ((0, "copy", 2), (1, "read", 1), (2, "write", 1)):
        best = (0.0, None)
        for grid in (1024, 2048, 4096, 16384, 65536, 262144):
            for unr in (1, 2, 4, 8):
                ms = L.cpk_ceiling_stream(kind, a.data_ptr(), b.data_ptr(), nbytes, grid, unr, s, reps)
                if ms > 0 and mult * nbytes / (ms * 1e-3) / 1e9 > best[0]:
                    best = (mult * nbytes / (ms * 1e-3) / 1e9, f"grid {grid} x 256, {unr} x 16 B in flight")
        out[name], cfg[name] = round(best[0], 1), best[1]
    nsteps = nbytes // (8 * 4096)
    best = (0.0, None)
    for grid in (1024, 2048, 4096, 16384, 65536):
        ms = L.cpk_ceiling_shaped(a.data_ptr(), b.data_ptr(), nsteps, 5, 8, grid, s, reps)
        if ms > 0 and 13 * 4096 * nsteps / (ms * 1e-3) / 1e9 > best[0]:
            best = (13 * 4096 * nsteps / (ms * 1e-3) / 1e9, f"grid {grid} x 256")
    out["decode_shaped"], cfg["decode_shaped"] = round(best[0], 1), best[1]
    torch.cuda.synchronize()
    del a, b
    torch.cuda.empty_cache()
    out["torch_copy"] = copy_ceiling(dev, nbytes)
    out["config"] = cfg
    return out


def dense_leg(args, dev, reps=10):
    """Decode from a DENSE packed stream (what arrives off a socket: unit starts at
    arbitrary byte offsets), headline size: sizes -> scan -> dense encode (untimed),
    then decode timed with HIP events on the launch stream."""
    n, ub = args.units, args.unit_bytes
    stream = torch.cuda.current_stream()
    d_in = cp.generate(n, ub, seed=args.seed, zero_thresh=args.zero_thresh, device=dev)
    in_off, in_len = cp.uniform_layout(n, ub, device=dev)
    lens = torch.empty(n, dtype=torch.int64, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    cp.encoded_size_batch(d_in, in_off, in_len, lens, st)
    off = cp.lengths_to_offsets(lens)
    P = int(off[-1].item())
    dense = torch.empty(P + 16, dtype=torch.uint8, device=dev)
    pk_off = off[:-1].contiguous()
    cp.encode_batch(d_in, in_off, in_len, dense, pk_off, lens, lens, st)
    d_out = torch.empty(n * ub, dtype=torch.uint8, device=dev)
    ulen = torch.zeros(n, dtype=torch.int64, device=dev)
    ust = torch.zeros(n, dtype=torch.int32, device=dev)
    run = lambda: cp.decode_batch(dense, pk_off, lens, d_out, in_off, in_len, ulen, ust, stream=stream)  # noqa: E731
    run()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record(stream)
    for _ in range(reps):
        run()
    ev[1].record(stream)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    ok = bool((ust == 0).all().item() and torch.equal(d_out, d_in))
    alg = n * ub + P + META_BYTES_PER_UNIT * n
    return {"decode_ms": round(ms, 4), "decode_GiB_s": round(n * ub / (ms * 1e-3) / 2 ** 30, 2),
            "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "packed_bytes": P, "bit_exact": ok,
            "note": "decode of 1M units from one dense packed stream (unaligned unit starts)"}


def host_path(args, dev, n_units=1 << 18, sweep=(4, 8, 16, 32, 64), nbuf=3):
    """PCIe-inclusive rates, reported beside the device-resident number and
    never as `value`. Host buffers are pinned; the batch (1 GiB unpacked) is cut into chunks
    pipelined over three streams, one per engine: H2D of chunk k+1, the kernels of chunk k and
    D2H of chunk k-1 run together (events order each chunk's three steps; a ring of `nbuf`
    device buffer sets, reused once their D2H is done). The chunk count is swept; the best
    count's rates are reported, with the sweep.
      decode: dense packed stream (P bytes) H2D -> decode -> unpacked D2H
      encode: unpacked H2D -> sizes -> scan -> dense encode -> packed D2H
    (the encode leg copies back each chunk's exact packed size, known here from a prior pass;
    a socket writer would read it from the sizes first)."""
    ub = args.unit_bytes
    d_all = cp.generate(n_units, ub, seed=args.seed, zero_thresh=args.zero_thresh, device=dev)
    in_off, in_len = cp.uniform_layout(n_units, ub, device=dev)
    lens = torch.empty(n_units, dtype=torch.int64, device=dev)
    st = torch.empty(n_units, dtype=torch.int32, device=dev)
    cp.encoded_size_batch(d_all, in_off, in_len, lens, st)
    off = cp.lengths_to_offsets(lens)
    dense = torch.empty(int(off[-1].item()) + 16, dtype=torch.uint8, device=dev)
    cp.encode_batch(d_all, in_off, in_len, dense, off[:-1].contiguous(), lens, lens, st)
    h_in = d_all.cpu().pin_memory()
    h_pk = dense.cpu().pin_memory()
    h_off = off.cpu()
    h_len = lens.cpu().pin_memory()
    h_out = torch.empty(n_units * ub, dtype=torch.uint8).pin_memory()
    h_pk2 = torch.empty_like(h_pk).pin_memory()
    del d_all, dense
    s_in, s_k, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))

    def run(name, chunks):
        per = n_units // chunks
        cmax = int((h_off[per::per] - h_off[:-1:per]).max().item()) + 16
        bufs = []
        for _ in range(nbuf):
            b = {"un": torch.empty(per * ub, dtype=torch.uint8, device=dev),
                 "pk": torch.empty(cmax, dtype=torch.uint8, device=dev),
                 "len": torch.empty(per, dtype=torch.int64, device=dev),
                 "olen": torch.empty(per, dtype=torch.int64, device=dev),
                 "st": torch.empty(per, dtype=torch.int32, device=dev),
                 "off": torch.empty(per + 1, dtype=torch.int64, device=dev),
                 "free": torch.cuda.Event()}
            b["u_off"], b["u_len"] = cp.uniform_layout(per, ub, device=dev)
            b["free"].record(s_out)
            bufs.append(b)

        def once():
            for c in range(chunks):
                b = bufs[c % nbuf]
                lo, hi = int(h_off[c * per]), int(h_off[(c + 1) * per])
                e_in, e_k = torch.cuda.Event(), torch.cuda.Event()
                s_in.wait_event(b["free"])  # chunk c - nbuf's D2H is done with this set
                with torch.cuda.stream(s_in):
                    if name == "decode":
                        b["pk"][:hi - lo].copy_(h_pk[lo:hi], non_blocking=True)
                        b["len"].copy_(h_len[c * per:(c + 1) * per], non_blocking=True)
                    else:
                        b["un"].copy_(h_in[c * per * ub:(c + 1) * per * ub], non_blocking=True)
                    e_in.record(s_in)
                s_k.wait_event(e_in)
                with torch.cuda.stream(s_k):
                    if name == "decode":
                        cp.lengths_to_offsets(b["len"], out=b["off"], stream=s_k)
                        cp.decode_batch(b["pk"], b["off"][:-1], b["len"], b["un"], b["u_off"], b["u_len"],
                                        b["olen"], b["st"], stream=s_k)
                    else:
                        cp.encoded_size_batch(b["un"], b["u_off"], b["u_len"], b["len"], b["st"], stream=s_k)
                        cp.lengths_to_offsets(b["len"], out=b["off"], stream=s_k)
                        cp.encode_batch(b["un"], b["u_off"], b["u_len"], b["pk"], b["off"], b["len"],
                                        b["olen"], b["st"], stream=s_k)
                    e_k.record(s_k)
                s_out.wait_event(e_k)
                with torch.cuda.stream(s_out):
                    if name == "decode":
                        h_out[c * per * ub:(c + 1) * per * ub].copy_(b["un"], non_blocking=True)
                    else:
                        h_pk2[lo:hi].copy_(b["pk"][:hi - lo], non_blocking=True)
                    b["free"].record(s_out)

        once()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            once()
        torch.cuda.synchronize(dev)
        rate = 3 * n_units * ub / (time.perf_counter() - t0) / 2 ** 30
        del bufs
        return rate

    res, table = {}, {}
    for name in ("decode", "encode"):
        rates = {c: run(name, c) for c in sweep}
        best = max(rates, key=rates.get)
        res[name + "_GiB_s"] = round(rates[best], 2)
        res[name + "_chunks"] = best
        table[name] = {str(c): round(r, 2) for c, r in rates.items()}
    res.update({"units": n_units, "unit_bytes": ub, "chunk_sweep_GiB_s": table,
                "bit_exact_roundtrip": bool(torch.equal(h_out, h_in) and
                                            torch.equal(h_pk2[:int(h_off[-1])], h_pk[:int(h_off[-1])])),
                "streams": 3, "buffer_sets": nbuf,
                "note": "GiB/s of unpacked bytes; pinned host buffers; H2D, kernels and D2H of different "
                        "chunks on three streams (PCIe Gen5 x16, 63 GB/s per direction spec)"})
    return res


def pareto_sizes(n, seed=0xC0DE0005):
    """unit size = 8 * floor(clamp(64 (1-u)^(-1/1.1), 64, 262144) / 8),
    a truncated Pareto (alpha = 1.1, mean ~424 B); u from a seeded numpy generator."""
    import numpy as np
    u = np.random.default_rng(seed).random(n)
    return (8 * np.floor(np.clip(64.0 * (1.0 - u) ** (-1.0 / 1.1), 64, 262144) / 8)).astype(np.int64)


def skewed_leg(args, dev, n=1 << 20, reps=10):
    """Config C5 (skewed sizes, p = 0.5): encode into capacity slots + decode from them,
    device-resident, HIP events on the launch stream. Reported beside `value`."""
    stream = torch.cuda.current_stream()
    sizes = torch.from_numpy(pareto_sizes(n)).to(dev)
    in_off = torch.zeros(n, dtype=torch.int64, device=dev)
    in_off[1:] = torch.cumsum(sizes, 0)[:-1]
    U = int(sizes.sum().item())
    d_in = cp.generate(1, U, seed=0xC0DE0005, zero_thresh=args.zero_thresh, device=dev)
    caps = (sizes // 8) * 10
    slots = (caps + 15) // 16 * 16
    pk_off = torch.zeros(n, dtype=torch.int64, device=dev)
    pk_off[1:] = torch.cumsum(slots, 0)[:-1]
    d_pk = torch.empty(int(slots.sum().item()), dtype=torch.uint8, device=dev)
    plen = torch.zeros(n, dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    d_out = torch.empty(U, dtype=torch.uint8, device=dev)
    ulen = torch.zeros(n, dtype=torch.int64, device=dev)
    ust = torch.zeros(n, dtype=torch.int32, device=dev)
    enc = lambda: cp.encode_batch(d_in, in_off, sizes, d_pk, pk_off, caps, plen, pst, stream=stream)  # noqa: E731
    dec = lambda: cp.decode_batch(d_pk, pk_off, plen, d_out, in_off, sizes, ulen, ust, stream=stream)  # noqa: E731
    enc()
    dec()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    torch.cuda.synchronize()
    t = [0.0, 0.0]
    for _ in range(reps):
        ev[0].record(stream)
        enc()
        ev[1].record(stream)
        dec()
        ev[2].record(stream)
        torch.cuda.synchronize()
        t[0] += ev[0].elapsed_time(ev[1])
        t[1] += ev[1].elapsed_time(ev[2])
    em, dm = t[0] / reps, t[1] / reps
    ok = bool((pst == 0).all().item() and (ust == 0).all().item() and torch.equal(ulen, sizes)
              and torch.equal(d_out, d_in))
    big = sizes > 4096
    P = int(plen.sum().item())
    alg = U + P + META_BYTES_PER_UNIT * n  # per direction, as the headline's roofline
    return {"units": n, "unpacked_bytes": U, "packed_bytes": P, "units_over_4KiB": int(big.sum().item()),
            "bytes_in_units_over_4KiB": int(sizes[big].sum().item()),
            "encode_ms": round(em, 4), "decode_ms": round(dm, 4), "alg_bytes": alg,
            "encode_frac": round(alg / (em * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "decode_frac": round(alg / (dm * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "GiB_s": round(U / ((em + dm) * 1e-3) / 2 ** 30, 2),
            "packed_ratio": round(int(plen.sum().item()) / U, 4), "bit_exact_roundtrip": ok,
            "note": "SURVEY config C5: truncated Pareto unit sizes 64 B..256 KiB, p = zero_thresh/256"}


def framer_leg(args, dev, conns=4096, msgs=16, reps=5):
    """SURVEY §8(f) row 3, RPC framer batching: `conns` connections, each with one socket
    read holding `msgs` packed 1-segment messages (framed 4096 B, p = zero_thresh/256).
    PackedConnections.handle_read pops every frame: one walk pass finds every held message
    of every connection and one decode pass frames them, H2D of the bytes and D2H of the frames
    included (a host-memory path: reported beside `value`, never as it). `ms` is the Python
    mirror's read; native_ms the capnp_packed_framer_read call a C / Zig caller makes on an
    assembled page-locked input (FramerSession.read_raw), assemble_ms the Python gathering of
    the per-connection bytes objects into such an input, readv_ms capnp_packed_framer_readv over
    the bytes objects themselves (the library's threaded gather; what handle_read uses)."""
    n = conns * msgs
    words = 511
    d_fr = cp.generate(n, 4096, seed=0xC0DE0007, zero_thresh=args.zero_thresh, device=dev)
    hdr = torch.tensor(list(struct.pack("<II", 0, words)), dtype=torch.uint8, device=dev)
    d_fr.view(n, 4096)[:, :8] = hdr
    off, ln = cp.uniform_layout(n, 4096, device=dev)
    slot = cp.encode_bound(4096)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    d_pk = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.zeros(n, dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    cp.encode_batch(d_fr, off, ln, d_pk, pk_off, pk_cap, plen, pst)
    torch.cuda.synchronize()
    pk_h, pl_h, fr_h = d_pk.cpu().numpy(), plen.cpu().numpy(), d_fr.cpu().numpy()
    streams = {c: b"".join(pk_h[i * slot:i * slot + int(pl_h[i])].tobytes() for i in range(c * msgs, (c + 1) * msgs))
               for c in range(conns)}
    packed_bytes = sum(len(v) for v in streams.values())
    # one long-lived session, as an event loop keeps it: the first read also pays the session's
    # device allocations (reported as first_read_ms), later reads of the same batch shape reuse them
    ok, first, all_ms, warm = True, None, [], []
    pc = cp.PackedConnections(conns, device=dev)
    # the share of each read spent in the native call (FramerSession.readv_raw) vs the views
    raw_ms, raw0 = [], pc.session.readv_raw

    def timed_raw(reads):
        t = time.perf_counter()
        r = raw0(reads)
        raw_ms.append(round((time.perf_counter() - t) * 1e3, 2))
        return r
    pc.session.readv_raw = timed_raw
    res = None
    for r in range(reps + 1):
        res = None  # the previous read's frames are handled and dropped before the next read
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = pc.handle_read(streams)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        all_ms.append(round(dt * 1e3, 2))
        if r == 0:
            first = dt
        else:
            warm.append(dt)
        for c in (0, conns // 2, conns - 1):
            fr = res[c]
            ok &= isinstance(fr, list) and len(fr) == msgs and all(
                fr[k] == fr_h[(c * msgs + k) * 4096:(c * msgs + k + 1) * 4096].tobytes() for k in range(msgs))
        ok &= all(isinstance(v, list) and len(v) == msgs for v in res.values())
    del res
    sess = pc.session
    del sess.readv_raw
    t0 = time.perf_counter()
    inp = sess.assemble(streams)
    asm = time.perf_counter() - t0
    nat_all = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        parts, status = sess.read_raw(*inp)
        dt = time.perf_counter() - t0
        if r > 0:
            nat_all.append(dt)
        ok &= sum(len(p[1]) for p in parts) == n and bool((status == cp.END_OF_STREAM).all())
        del parts
    rv_all = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        parts, status = sess.readv_raw(streams)
        dt = time.perf_counter() - t0
        if r > 0:
            rv_all.append(dt)
        ok &= sum(len(p[1]) for p in parts) == n and bool((status == cp.END_OF_STREAM).all())
        del parts
    med = statistics.median(warm)
    nat, rv = statistics.median(nat_all), statistics.median(rv_all)
    return {"connections": conns, "messages_per_read": msgs, "framed_bytes": 4096, "packed_bytes": packed_bytes,
            "ms": round(med * 1e3, 2), "framed_GiB_s": round(n * 4096 / med / 2 ** 30, 2),
            "frames_per_s": round(n / med), "best_ms": round(min(warm) * 1e3, 2),
            "first_read_ms": round(first * 1e3, 2), "reads_ms": all_ms, "reads_readv_ms": raw_ms,
            "native_ms": round(nat * 1e3, 2), "native_framed_GiB_s": round(n * 4096 / nat / 2 ** 30, 2),
            "readv_ms": round(rv * 1e3, 2), "assemble_ms": round(asm * 1e3, 2), "bit_exact": bool(ok),
            "note": "host buffers in and out (PCIe + host-side framing); one framer session; ms, native_ms and "
                    "readv_ms are medians of the reads after the first (first_read_ms includes the session's "
                    "device allocations), best_ms the fastest warm read"}


def framer_split_leg(args, dev, read_bytes=65536, sizes_words=(1 << 17, 1 << 19, 1 << 21, 1 << 23)):
    """Verdict r3 item 2, RPC framing of packed messages that span socket reads: one
    connection receives one message of 1, 4, 16 and 64 MiB framed (the last is the 8 Mi-word
    limit, framing.zig:5) in 64 KiB reads (connection.zig:68's read size) through
    PackedConnections (the device-resident FramerSession). Time from the first
    read to the popped frame, host buffers in and out; bytes uploaded against the stream.
    Linear when ms per MiB stays flat as the message grows."""
    rows = []
    for words in sizes_words:
        fb = 8 * words
        d_fr = cp.generate(1, fb, seed=0xC0DE000B, zero_thresh=args.zero_thresh, device=dev)
        d_fr[:8] = torch.tensor(list(struct.pack("<II", 0, words - 1)), dtype=torch.uint8, device=dev)
        off, ln = cp.uniform_layout(1, fb, device=dev)
        slot = cp.encode_bound(fb)
        pk_off, pk_cap = cp.uniform_layout(1, slot, device=dev)
        d_pk = torch.zeros(slot, dtype=torch.uint8, device=dev)
        plen = torch.zeros(1, dtype=torch.int64, device=dev)
        pst = torch.zeros(1, dtype=torch.int32, device=dev)
        cp.encode_batch(d_fr, off, ln, d_pk, pk_off, pk_cap, plen, pst)
        torch.cuda.synchronize()
        stream = d_pk[:int(plen.item())].cpu().numpy().tobytes()
        reads = [stream[i:i + read_bytes] for i in range(0, len(stream), read_bytes)]
        pc = cp.PackedConnections(1, device=dev)
        frames = []
        t0 = time.perf_counter()
        for piece in reads:
            res = pc.handle_read({0: piece})
            frames += res.get(0, []) if isinstance(res.get(0), list) else [res.get(0)]
        dt = time.perf_counter() - t0
        ok = len(frames) == 1 and isinstance(frames[0], memoryview) and bytes(frames[0]) == d_fr.cpu().numpy().tobytes()
        st = pc.session.stats()
        rows.append({"framed_MiB": fb / 2 ** 20, "packed_bytes": len(stream), "reads": len(reads),
                     "ms": round(dt * 1e3, 2), "ms_per_MiB": round(dt * 1e3 / (fb / 2 ** 20), 3),
                     "framed_GiB_s": round(fb / dt / 2 ** 30, 3),
                     "uploaded_over_stream": round(st["uploaded_bytes"] / len(stream), 4),
                     "moved_over_stream": round(st["moved_bytes"] / len(stream), 4), "bit_exact": bool(ok)})
        del d_fr, d_pk
        torch.cuda.empty_cache()
    return {"read_bytes": read_bytes, "rows": rows,
            "note": "one message per connection in 64 KiB reads, host buffers in and out; the walk resumes "
                    "across reads (capnp_packed_framer_*), so ms_per_MiB flat = linear"}


def message_leg(args, dev, reps=10, segs=4, seg_words=127):
    """SURVEY §8(f) row 2, framing fused with the codec: 1M messages of 4 segments x
    127 words (framed 4088 B) from a segment pool, packed straight from the segment
    lists (encode_message_batch), against toBytes as a device gather + encode_batch;
    then Message.init on device (message_init_batch) over the decoded frames.
    Reported beside `value`, never as it."""
    n = args.units
    stream = torch.cuda.current_stream()
    sb = 8 * seg_words
    pool = cp.generate(n * segs, sb, seed=0xC0DE0006, zero_thresh=args.zero_thresh, device=dev)
    seg_ptr = pool.data_ptr() + torch.arange(n * segs, dtype=torch.int64, device=dev) * sb
    seg_len = torch.full((n * segs,), sb, dtype=torch.int64, device=dev)
    first = torch.arange(0, n * segs, segs, dtype=torch.int32, device=dev)
    count = torch.full((n,), segs, dtype=torch.int32, device=dev)
    hw = (1 + segs + (0 if segs % 2 else 1)) // 2
    fb = 8 * hw + segs * sb
    slot = (cp.encode_bound(fb) + 15) // 16 * 16
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    pk_cap.fill_(cp.encode_bound(fb))
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.zeros(n, dtype=torch.int64, device=dev)
    pst = torch.zeros(n, dtype=torch.int32, device=dev)
    # toBytes materialised: header words + segment copy, then encode_batch (the unfused path)
    framed = torch.empty(n * fb, dtype=torch.uint8, device=dev)
    hdr = torch.zeros(2 * hw, dtype=torch.int32, device=dev)
    hdr[0] = segs - 1
    hdr[1:1 + segs] = seg_words
    f_off, f_len = cp.uniform_layout(n, fb, device=dev)
    plen2 = torch.zeros_like(plen)
    fv = framed.view(n, fb)

    def fused():
        cp.encode_message_batch(seg_ptr, seg_len, first, count, d_pk, pk_off, pk_cap, plen, pst, stream=stream)

    def unfused():
        fv[:, :8 * hw].copy_(hdr.view(torch.uint8).expand(n, 8 * hw))
        fv[:, 8 * hw:].copy_(pool.view(n, segs * sb))
        cp.encode_batch(framed, f_off, f_len, d_pk, pk_off, pk_cap, plen2, pst, stream=stream)

    def timed(fn):
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps

    t_unfused = timed(unfused)
    ok = bool((pst == 0).all().item())
    t_fused = timed(fused)
    ok = ok and bool((pst == 0).all().item() and torch.equal(plen, plen2))
    # decode the packed messages and parse their segment tables on device
    d_out = torch.empty(n * fb, dtype=torch.uint8, device=dev)
    ulen = torch.zeros(n, dtype=torch.int64, device=dev)
    ust = torch.zeros(n, dtype=torch.int32, device=dev)
    cp.decode_batch(d_pk, pk_off, plen, d_out, f_off, f_len, ulen, ust, stream=stream)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    so = torch.zeros(n * segs, dtype=torch.int64, device=dev)
    sl = torch.zeros(n * segs, dtype=torch.int64, device=dev)
    mst = torch.zeros(n, dtype=torch.int32, device=dev)
    t_init = timed(lambda: cp.message_init_batch(d_out, f_off, f_len, segs, cnt, so, sl, mst, stream=stream))
    ok = ok and bool(torch.equal(d_out, framed) and (mst == 0).all().item() and (cnt == segs).all().item()
                     and (sl == sb).all().item())
    P = int(plen.sum().item())
    # encode: the segment words + headers out of the pool, P written, per-message metadata
    # (segment pointer / length / first / count and the slot arrays) ~ 44 B + 20 B per segment
    alg = n * fb + P + (META_BYTES_PER_UNIT + 20 * segs) * n
    return {"messages": n, "segments_per_message": segs, "framed_bytes": fb, "packed_bytes": P,
            "fused_encode_ms": round(t_fused, 4), "tobytes_copy_plus_encode_ms": round(t_unfused, 4),
            "alg_bytes": alg, "encode_frac": round(alg / (t_fused * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "fused_GiB_s": round(n * fb / (t_fused * 1e-3) / 2 ** 30, 2),
            "message_init_ms": round(t_init, 4), "bit_exact": ok,
            "note": "GiB/s of framed bytes; fused = encode_message_batch from segment lists (no framed copy)"}


def read_message_leg(args, dev, reps=10):
    """SURVEY §8(f) row 1, Reader.readPackedMessage (reader.zig:84-156) batched: the
    same 1M x 4 KiB units made into framed messages (one segment of 511 words), packed
    into slots, then read back one message per reader stream, each stream holding its
    message plus 8 bytes of whatever follows. Device-resident, HIP events on the
    launch stream; reported beside `value`, never as it."""
    n, ub = args.units, args.unit_bytes
    stream = torch.cuda.current_stream()
    wl = Workload(n, ub, args.seed, args.zero_thresh, unit_base=0, dev=dev)
    wl.d_in.view(torch.int64).view(n, ub // 8)[:, 0] = (ub // 8 - 1) << 32  # segment table
    wl.encode(stream)
    used = torch.zeros(n, dtype=torch.int64, device=dev)
    tail = torch.minimum(wl.plen + 8, wl.pk_cap)

    def run():
        cp.read_message_batch(wl.d_pk, wl.pk_off, tail, wl.d_out, wl.in_off, wl.in_len, wl.ulen, used, wl.ust,
                              stream=stream)

    run()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record(stream)
    for _ in range(reps):
        run()
    ev[1].record(stream)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    ok = bool((wl.ust == 0).all().item() and torch.equal(used, wl.plen) and torch.equal(wl.d_out, wl.d_in))
    P = int(wl.plen.sum().item())
    alg = n * ub + P + META_BYTES_PER_UNIT * n + 8 * n  # + consumed (8 B per stream)
    return {"ms": round(ms, 4), "GiB_s": round(n * ub / (ms * 1e-3) / 2 ** 30, 2),
            "alg_bytes": alg, "alg_GB_s": round(alg / (ms * 1e-3) / 1e9, 1),
            "decode_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "messages": n, "framed_bytes": ub, "bit_exact": ok,
            "note": "GiB/s of framed (unpacked) bytes; header pass + framed-length walk + indexed decode"}


def validate_leg(args, dev, reps=10, n=1 << 20, distinct=4096, cpu_s=3.0):
    """SURVEY §8(f) row 4, Message.validate (message.zig:699-969) batched, with the
    default ValidationOptions (:331-335), on two device-resident corpora:
      trees: 1M framed messages, `distinct` random valid trees (tests/msggen.py: 1-4
             segments, structs, lists of every element size, pointer lists, inline-
             composite lists, single and double far pointers, depth <= 6) repeated;
      c1:    256K copies of the reference bench's own 20,536-B message.
    Algorithmic bytes = the words the walk reads (pointer slots, landing pads, tags:
    msggen's per-tree count) x 8 + the segment table + 24 B of per-message metadata.
    CPU side: the oracle's recursive restatement, one thread, on the distinct trees."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import numpy as np
    import msggen
    import pyref
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(0xC0DE0008)
    trees = [msggen.RandomTree(rng) for _ in range(distinct)]
    msgs = [t.framed() for t in trees]
    lens = np.array([len(m) for m in msgs], dtype=np.int64)
    alg_one = np.array([8 * t.reads + msggen.header_bytes(m) + 24 for t, m in zip(trees, msgs)], dtype=np.int64)
    base = torch.from_numpy(np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()).to(dev)
    reps_n = n // distinct
    d_in = base.repeat(reps_n)
    off1 = np.zeros(distinct, dtype=np.int64)
    off1[1:] = np.cumsum(lens)[:-1]
    offs = (torch.from_numpy(off1).to(dev)[None, :] + (torch.arange(reps_n, device=dev) * int(lens.sum()))[:, None])
    in_off = offs.reshape(-1).contiguous()
    in_len = torch.from_numpy(lens).to(dev).repeat(reps_n)
    st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    words = torch.zeros(n, dtype=torch.int64, device=dev)

    def timed(fn):
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps

    ms = timed(lambda: cp.validate_batch(d_in, in_off, in_len, st, words, stream=stream))
    w2 = words.view(reps_n, distinct)
    ok = bool((st == 0).all().item() and (w2 == w2[0:1]).all().item())
    alg = int(alg_one.sum()) * reps_n
    reads = sum(t.reads for t in trees) * reps_n
    out = {"trees": {"messages": n, "distinct": distinct, "framed_bytes": int(lens.sum()) * reps_n,
                     "pointer_words_read": reads, "ms": round(ms, 4),
                     "messages_per_s": round(n / (ms * 1e-3)), "words_read_per_s": round(reads / (ms * 1e-3)),
                     "alg_GB_s": round(alg / (ms * 1e-3) / 1e9, 1),
                     "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "all_valid": ok}}
    del d_in, in_off, in_len, st, words, offs
    torch.cuda.empty_cache()
    # the reference bench's message (one segment: root struct -> text + u64 list)
    c1 = pyref.frame(pyref.bench_message_segments())
    n1 = 1 << 18
    d1 = torch.from_numpy(np.frombuffer(c1, dtype=np.uint8).copy()).to(dev).repeat(n1)
    o1, l1 = cp.uniform_layout(n1, len(c1), device=dev)
    s1 = torch.full((n1,), -1, dtype=torch.int32, device=dev)
    wd1 = torch.zeros(n1, dtype=torch.int64, device=dev)
    ms1 = timed(lambda: cp.validate_batch(d1, o1, l1, s1, wd1, stream=stream))
    ok1 = bool((s1 == 0).all().item() and (wd1 == wd1[0]).all().item())
    out["c1"] = {"messages": n1, "framed_bytes": len(c1), "ms": round(ms1, 4),
                 "messages_per_s": round(n1 / (ms1 * 1e-3)),
                 "validated_GiB_s": round(n1 * len(c1) / (ms1 * 1e-3) / 2 ** 30, 1),
                 "traversal_words": int(wd1[0].item()), "all_valid": ok1}
    del d1
    torch.cuda.empty_cache()
    # CPU: the oracle walk on the distinct trees, one thread
    import oracle
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < cpu_s:
        for m in msgs:
            oracle.validate(m)
        done += len(msgs)
    el = time.perf_counter() - t0
    out["cpu_oracle_1core_trees"] = {"messages_per_s": round(done / el), "sample": f"{done} tree validations",
                                     "note": "includes a ctypes call per message (~1 us)"}
    out["note"] = ("device: lane per message, LDS stack of pointer runs; alg bytes = walked words x 8 + "
                   "segment table + 24 B metadata per message")
    return out


def load_traffic(config_key):
    """PMC HBM bytes per launch for this config (scripts/pmc_traffic.py output)."""
    path = os.environ.get("CPK_TRAFFIC_JSON") or os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(config_key)
    except Exception:
        return None


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """One child process per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set), started
    before this process touches any GPU; rank 0 prints the JSON line. Returns the
    worst exit status."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every rank: when one fails, the others would block in their collectives, so
    # they are terminated (then killed after a grace period) and the failure is returned
    failed = None
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            failed = bad[0]
            break
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.time() + 15
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return failed


def dry_run(args, world, rank):
    """CPU rehearsal of the multi-rank step (gloo): each rank packs its shard of a small
    batch with the oracle, then the same all-gather of packed totals as the GPU step."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import oracle
    if world > 1:
        dist.init_process_group("gloo")
    n, ub = args.units, args.unit_bytes
    data = oracle.generate(n, ub, seed=args.seed, zero_thresh=args.zero_thresh, unit_base=rank * n)
    t0 = time.perf_counter()
    local = sum(len(oracle.pack(data[i * ub:(i + 1) * ub].tobytes())[1]) for i in range(n))
    totals = sharding.gather_packed_totals(local)
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "dry run (CPU oracle, gloo): per-rank pack + all-gather of packed totals",
                          "n_gpus": world, "dry_run": True, "units_per_rank": n, "unit_bytes": ub,
                          "packed_totals": totals.tolist(), "packed_total_all_ranks": int(totals.sum().item()),
                          "shard_offsets": [sharding.shard_byte_offset(totals, r) for r in range(world)],
                          "seconds": round(float(el.item()), 4)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def measure(wl, args, steps, warmup, world, dev):
    """Time `steps` steps of one workload; roofline of encode and decode on their own."""
    n, ub = wl.n, wl.ub
    elapsed, enc_ms, dec_ms, gathered = time_steps(wl, steps, warmup, world, dev)
    P = int(wl.plen.sum().item())
    alg = n * ub + P + META_BYTES_PER_UNIT * n  # per launch on one GPU, same for encode and decode
    return {"elapsed": elapsed, "enc_ms": enc_ms, "dec_ms": dec_ms, "gathered": gathered, "P": P, "alg": alg,
            "ok": wl.verify(),
            "encode_frac": alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "decode_frac": alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run and os.environ.get("CPK_DRY_RUN_FAIL_RANK") == str(rank):
        sys.exit(3)  # test hook (tests/test_bench_launcher.py): a rank that dies before the rendezvous
    if args.dry_run:
        if args.units == 1 << 20:
            args.units = 64
        return dry_run(args, world, rank)
    if args.same_gpu:
        local = 0
    if world > 1 and args.same_gpu:
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    if args.decoder:
        cp.set_decoder(args.decoder)
    if args.only:
        legs = {"validate": validate_leg, "c5": skewed_leg, "dense": dense_leg, "read_message": read_message_leg,
                "framing": message_leg, "rpc_framer": framer_leg, "rpc_framer_split": framer_split_leg,
                "host_path": host_path}
        print(json.dumps({args.only: legs[args.only](args, dev)}), flush=True)
        return
    n, ub = args.units, args.unit_bytes
    wl = Workload(n, ub, args.seed, args.zero_thresh, unit_base=rank * n, dev=dev)
    head = measure(wl, args, args.steps, args.warmup, world, dev)
    ok_t = torch.tensor([1 if head["ok"] else 0], device="cpu" if _host_collectives() else dev)
    if world > 1:
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
    packed_all = int(head["gathered"].sum().item())
    elapsed, enc_ms, dec_ms = head["elapsed"], head["enc_ms"], head["dec_ms"]

    def sweep_entry(m, thr, steps):
        return {"zero_thresh": thr, "GiB_s": round(world * n * ub / (m["elapsed"] / steps) / 2 ** 30, 2),
                "encode_ms": round(m["enc_ms"], 4), "decode_ms": round(m["dec_ms"], 4),
                "encode_frac": round(m["encode_frac"], 4), "decode_frac": round(m["decode_frac"], 4),
                "packed_ratio": round(m["P"] / (n * ub), 4), "bit_exact_roundtrip": m["ok"]}

    extra = {}
    if world == 1:
        extra["sweep"] = {"p0.5": sweep_entry(head, args.zero_thresh, args.steps)}
        if not args.no_sweep:
            for thr, name in ((26, "p0.1"), (230, "p0.9")):
                del wl
                torch.cuda.empty_cache()
                wl = Workload(n, ub, args.seed, thr, unit_base=rank * n, dev=dev)
                k = max(5, args.steps // 2)
                extra["sweep"][name] = sweep_entry(measure(wl, args, k, 2, world, dev), thr, k)
        del wl
        torch.cuda.empty_cache()
        if not args.no_ceilings:
            extra["roofline_ceilings_GBps"] = ceilings(dev, n * ub)
        if not args.no_dense:
            torch.cuda.empty_cache()
            extra["dense_stream"] = dense_leg(args, dev)
        if not args.no_read_message:
            torch.cuda.empty_cache()
            extra["read_message"] = read_message_leg(args, dev)
            torch.cuda.empty_cache()
            extra["message_framing"] = message_leg(args, dev)
        if not args.no_read_message:
            # before C5 (the framer's first reads in a bench process sometimes run
            # 2x slower, cause open; reads_ms shows which case a run hit)
            torch.cuda.empty_cache()
            extra["rpc_framer"] = framer_leg(args, dev)
            torch.cuda.empty_cache()
            extra["rpc_framer_split"] = framer_split_leg(args, dev)
        if not args.no_skewed:
            torch.cuda.empty_cache()
            extra["c5_skewed"] = skewed_leg(args, dev)
        if not args.no_validate:
            torch.cuda.empty_cache()
            extra["validate"] = validate_leg(args, dev)
        if not args.no_c1:
            extra["c1_bench_message"] = c1_leg()

    if rank == 0:
        steps = args.steps
        ms_per_step = elapsed / steps * 1e3
        U_total = world * n * ub
        value = U_total / (elapsed / steps) / 2 ** 30
        alg_bytes = head["alg"]
        role, dom_ms = ("decode", dec_ms) if dec_ms >= enc_ms else ("encode", enc_ms)
        achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
        cfg_key = f"{n}x{ub}_t{args.zero_thresh}"
        prof = (load_traffic(cfg_key) or {}).get(role) or {}
        traffic = prof.get("total_bytes")
        dom = ", ".join(prof.get("kernels", [])) or role
        line = {
            "metric": "GiB/s device-resident packed encode+decode, 1M x 4KiB segments",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device counter-hash generator, DESIGN.md §4)",
            "config": {"workload": f"{n} units x {ub} B per GPU, zero-byte p={args.zero_thresh}/256, "
                                   "encode into capacity slots + decode from slots",
                       "units_per_gpu": n, "unit_bytes": ub, "zero_thresh": args.zero_thresh,
                       "parallelism": f"shard{world}"},
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
                         "encode_frac": round(head["encode_frac"], 4), "decode_frac": round(head["decode_frac"], 4),
                         "ceilings_GBps": extra.pop("roofline_ceilings_GBps", None)},
            "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_GiB_s": round(n * ub / (enc_ms * 1e-3) / 2 ** 30, 2),
            "decode_GiB_s": round(n * ub / (dec_ms * 1e-3) / 2 ** 30, 2),
            "packed_ratio": round(packed_all / U_total, 4),
            "packed_total_all_ranks": packed_all,
            "bit_exact_roundtrip": bool(ok_t.item()),
        }
        line.update(extra)
        ceil = line["roofline"].get("ceilings_GBps")
        if ceil:  # the dominant kernel against what this box's HBM delivers for its traffic shape
            shaped = ceil.get("decode_shaped") if role == "decode" else ceil.get("copy")
            if shaped:
                line["roofline"]["frac_of_box_ceiling"] = round(achieved / shaped, 4)
        if args.same_gpu and world > 1:
            line["same_gpu_rehearsal"] = {"ranks": world, "devices": 1, "collectives": "gloo",
                                          "note": "all ranks share cuda:0: checks the N-rank step, not a scaling number"}
        if world == 1 and not args.no_host_path:
            line["host_path"] = host_path(args, dev)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
