"""Multi-GPU sharding of a batch of independent units.

Units are independent packPacked / unpackPacked calls, so a batch shards with no
data exchange: rank r owns units [r*N/W, (r+1)*N/W). The only collective is an
all-gather of each rank's packed total (one int64 per rank, RCCL over xGMI with
the "nccl" backend, gloo on CPU), which gives every rank the global byte offset
of its shard in a dense cross-rank packed stream and the job-wide packed size.
The payload never crosses GPUs.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(rank: int, world: int, n_units: int) -> tuple[int, int]:
    """Contiguous, balanced shard [lo, hi) of n_units for rank (sizes differ by <= 1)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    q, r = divmod(n_units, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def gather_packed_totals(local_total, group=None, collective_at_world1: bool = False) -> torch.Tensor:
    """All-gather each rank's packed byte total. `local_total` is an int or a
    0-d/1-element int64 tensor (device tensor for RCCL, CPU tensor for gloo).
    Returns a (world,) int64 tensor on the same device. A world of one is a copy
    unless `collective_at_world1` (the test that puts RCCL's all-gather on the GPU,
    tests/test_gpu_rccl.py)."""
    if isinstance(local_total, torch.Tensor):
        t = local_total.reshape(1).to(torch.int64)
    else:
        dev = torch.device("cuda", torch.cuda.current_device()) if (
            dist.is_initialized() and dist.get_backend(group) == "nccl") else torch.device("cpu")
        t = torch.tensor([int(local_total)], dtype=torch.int64, device=dev)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    out = torch.empty(world, dtype=torch.int64, device=t.device)
    if world == 1 and not (collective_at_world1 and dist.is_initialized()):
        out.copy_(t)
    else:
        dist.all_gather_into_tensor(out, t, group=group)
    return out


def shard_byte_offset(totals: torch.Tensor, rank: int) -> int:
    """Global byte offset of rank's shard in the concatenated packed stream."""
    return int(totals[:rank].sum().item())
