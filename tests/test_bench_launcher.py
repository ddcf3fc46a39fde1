"""bench.py's multi-rank launcher on the CPU (gloo): `bench.py --gpus 2 --dry-run`
starts two rank processes itself (RANK / WORLD_SIZE / MASTER_* set, nothing touches a
GPU), each packs its shard with the oracle and all-gathers its packed total, exactly
the collective of the GPU step. The totals must equal a
single-process computation over the same global units."""
import json
import os
import subprocess
import sys

import pytest

import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", *extra], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints the only JSON line
    return json.loads(lines[0])


def test_launcher_two_ranks_all_gather():
    n, ub, seed, thr = 48, 1024, 0xC0DE0009, 128
    res = _run("--gpus", "2", "--units", str(n), "--unit-bytes", str(ub), "--seed", str(seed))
    assert res["n_gpus"] == 2 and res["dry_run"]
    data = oracle.generate(2 * n, ub, seed=seed, zero_thresh=thr)
    lens = [len(oracle.pack(data[i * ub:(i + 1) * ub].tobytes())[1]) for i in range(2 * n)]
    assert res["packed_totals"] == [sum(lens[:n]), sum(lens[n:])]
    assert res["shard_offsets"] == [0, sum(lens[:n])]
    assert res["packed_total_all_ranks"] == sum(lens)


def test_launcher_eight_ranks_all_gather():
    """World size 8, the driver's scaling run: ranks, shard offsets and the
    job-wide packed total from the all-gather, against one process packing all 8 shards."""
    n, ub, seed, thr, world = 24, 512, 0xC0DE0019, 128, 8
    res = _run("--gpus", str(world), "--units", str(n), "--unit-bytes", str(ub), "--seed", str(seed))
    assert res["n_gpus"] == world and res["dry_run"] and res["units_per_rank"] == n
    data = oracle.generate(world * n, ub, seed=seed, zero_thresh=thr)
    lens = [len(oracle.pack(data[i * ub:(i + 1) * ub].tobytes())[1]) for i in range(world * n)]
    per = [sum(lens[r * n:(r + 1) * n]) for r in range(world)]
    assert res["packed_totals"] == per
    assert res["shard_offsets"] == [sum(per[:r]) for r in range(world)]
    assert res["packed_total_all_ranks"] == sum(lens)


def test_launcher_eight_ranks_one_fails():
    """A rank of eight that dies before the rendezvous: the launcher stops the other seven
    (they would wait in the rendezvous) and returns the failed rank's status."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CPK_DRY_RUN_FAIL_RANK"] = "5"
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--gpus", "8", "--units", "8"],
                         env=env, capture_output=True, text=True, timeout=200)
    assert out.returncode == 3, out.stderr[-2000:]
    assert time.time() - t0 < 150


def test_launcher_single_rank():
    res = _run("--units", "16", "--unit-bytes", "512")
    assert res["n_gpus"] == 1 and len(res["packed_totals"]) == 1


def test_launcher_stops_the_other_ranks_when_one_fails():
    # rank 1 exits before the rendezvous: rank 0 would wait in it for 30 minutes; the
    # launcher notices, terminates rank 0 and returns rank 1's status
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CPK_DRY_RUN_FAIL_RANK"] = "1"
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--gpus", "2", "--units", "8"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 3, out.stderr[-2000:]
    assert time.time() - t0 < 90


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_same_gpu_rehearsal_eight_ranks_64k_units():
    """The N = 8 GPU step rehearsed on one card (bench.py --gpus 8 --same-gpu): eight ranks,
    64K x 4 KiB units each on cuda:0 with the HIP library, bit-exact round trips, and the
    all-gathered job-wide packed total equal to the oracle's over the same 512K global units."""
    n, ub, seed, thr, world = 1 << 16, 4096, 0xC0DE001A, 128, 8
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", str(world), "--same-gpu",
                          "--units", str(n), "--seed", str(seed), "--steps", "2", "--warmup", "1"],
                         env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["bit_exact_roundtrip"] and res["same_gpu_rehearsal"]["ranks"] == world
    import numpy as np
    data = oracle.generate(world * n, ub, seed=seed, zero_thresh=thr, threads=16)
    off = np.arange(world * n + 1, dtype=np.uint64) * ub
    pk_off = np.arange(world * n + 1, dtype=np.uint64) * (10 * ub // 8)
    _, plen, st = oracle.pack_batch(data, off, pk_off, threads=16)
    assert (st == 0).all()
    assert res["packed_total_all_ranks"] == int(plen.sum())


@pytest.mark.gpu
def test_same_gpu_rehearsal_two_ranks():
    # the N-rank GPU step (bench.py --gpus 2 --same-gpu): both ranks code their own units
    # on cuda:0 with the HIP library, bit-exact, and all-gather their packed totals; the
    # gathered total must equal the oracle's over the same global units
    n, ub, seed, thr = 512, 4096, 0xC0DE000A, 128
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--same-gpu",
                          "--units", str(n), "--seed", str(seed), "--steps", "2", "--warmup", "1"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["bit_exact_roundtrip"] and res["same_gpu_rehearsal"]["devices"] == 1
    data = oracle.generate(2 * n, ub, seed=seed, zero_thresh=thr)
    total = sum(len(oracle.pack(data[i * ub:(i + 1) * ub].tobytes())[1]) for i in range(2 * n))
    assert res["packed_total_all_ranks"] == total
