"""RCCL on the GPU: a fresh process initialises torch.distributed
with the "nccl" backend (RCCL on ROCm) at world size 1 before any GPU call, as bench.py's ranks
do, encodes a batch through the C-ABI on its GPU, and all-gathers its device-resident packed
total with all_gather_into_tensor (sharding.gather_packed_totals, the collective forced at world
1). The gathered total must equal the sum of the per-unit packed lengths, on the device, and the
process must tear the group down cleanly. N > 1 is the driver's 8-GPU run; the gloo tests
(tests/test_sharding.py, tests/test_bench_launcher.py) cover the multi-rank logic on CPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "capnp-zig_amd"))
import torch
import torch.distributed as dist
dist.init_process_group("nccl", rank=0, world_size=1)   # before any GPU call
try:
    torch.cuda.set_device(0)
    import capnp_packed as cp
    import sharding
    n, ub = 4096, 4096
    dev = torch.device("cuda", 0)
    d_in = cp.generate(n, ub, seed=0xC0DE0005, zero_thresh=128, device=dev)
    in_off, in_len = cp.uniform_layout(n, ub, device=dev)
    slot = cp.encode_bound(ub)
    pk_off, pk_cap = cp.uniform_layout(n, slot, device=dev)
    d_pk = torch.empty(n * slot, dtype=torch.uint8, device=dev)
    plen = torch.empty(n, dtype=torch.int64, device=dev)
    pst = torch.empty(n, dtype=torch.int32, device=dev)
    cp.encode_batch(d_in, in_off, in_len, d_pk, pk_off, pk_cap, plen, pst)
    local = plen.sum().reshape(1)
    totals = sharding.gather_packed_totals(local, collective_at_world1=True)
    torch.cuda.synchronize()
    print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(),
                      "device": str(totals.device), "total": int(totals[0].item()),
                      "expect": int(plen.cpu().sum().item()), "status_ok": int((pst == 0).all().item()),
                      "offset": sharding.shard_byte_offset(totals, 0)}), flush=True)
finally:
    dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_all_gather_of_packed_totals_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    got = json.loads(line)
    assert got["backend"] == "nccl" and got["world"] == 1 and got["device"].startswith("cuda")
    assert got["status_ok"] == 1 and got["total"] == got["expect"] > 0 and got["offset"] == 0
