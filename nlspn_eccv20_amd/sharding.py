"""Batch sharding for multi-GPU inference.

Each image's propagation depends only on that image, so a batch splits across
ranks with no exchange step — the MI355X form of the reference's
nn.DataParallel dim-0 scatter (src/main.py:366).  No collective touches the data
path; `max_over_ranks` is only for timing (bench.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, stop) of the batch owned by `rank`; chunk sizes as
    torch.chunk / DataParallel scatter (ceil(batch/world), trailing ranks may get less)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} for world {world}")
    step = -(-batch // world)
    start = min(batch, rank * step)
    return start, min(batch, start + step)


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
