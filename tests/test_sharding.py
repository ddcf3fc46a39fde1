"""Multi-process (gloo, world_size 2, CPU) test of the sharding path.

Each rank packs its shard with the oracle (CPU stand-in for the per-rank GPU
encode; the GPU path is covered by the gpu tests), all-gathers its packed total,
and checks offsets/totals against a single-process computation.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import sharding

N_UNITS, UNIT, SEED, THR = 37, 512, 0xC0DE0004, 128


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _expected_lengths():
    import oracle
    data = oracle.generate(N_UNITS, UNIT, seed=SEED, zero_thresh=THR)
    return [len(oracle.pack(data[i * UNIT:(i + 1) * UNIT].tobytes())[1]) for i in range(N_UNITS)]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        lo, hi = sharding.shard_range(rank, world, N_UNITS)
        data = oracle.generate(hi - lo, UNIT, seed=SEED, zero_thresh=THR, unit_base=lo)
        local = sum(len(oracle.pack(data[i * UNIT:(i + 1) * UNIT].tobytes())[1]) for i in range(hi - lo))
        totals = sharding.gather_packed_totals(local)
        q.put((rank, lo, hi, local, totals.tolist(), sharding.shard_byte_offset(totals, rank)))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions_exactly():
    for n in (0, 1, 7, 64, 1000003):
        for w in (1, 2, 3, 8):
            ranges = [sharding.shard_range(r, w, n) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        sharding.shard_range(2, 2, 10)


def test_gloo_world2_all_gather_of_packed_totals():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lens = _expected_lengths()
    totals = results[0][4]
    assert results[1][4] == totals
    for rank, lo, hi, local, _, off in results:
        assert local == sum(lens[lo:hi])
        assert off == sum(lens[:lo])
    assert sum(totals) == sum(lens)
    assert np.all(np.array(totals) > 0)
