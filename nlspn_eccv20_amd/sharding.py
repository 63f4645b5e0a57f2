"""Batch sharding for multi-GPU inference.

Each image's propagation depends only on that image, so a batch splits across
ranks (or devices) with no exchange step — the MI355X form of the reference's
nn.DataParallel dim-0 scatter (src/main.py:366).  No collective touches the data
path; `max_over_ranks` / `gather_over_ranks` are only for timing (bench.py).

  shard_range       — [start, stop) of a batch owned by one rank
  propagate_sharded — one process, several GPUs: scatter a batch over devices,
                      run propagate() on each device's current stream, gather
"""
from __future__ import annotations

from typing import Optional, Sequence

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


def gather_over_ranks(x: float, device=None) -> list:
    """Every rank's value of a scalar (timing spread), in rank order."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def propagate_sharded(pred_init, dep, confidence, aff, offset, gamma, devices: Sequence, **kw) -> dict:
    """propagate() over a batch scattered across `devices` (dim 0, shard_range sizes),
    one device per shard, results gathered onto pred_init's device — DataParallel's
    scatter/gather without replicating any module (the section has no weights but γ,
    which is copied to each device).  The shards run concurrently: every launch is
    asynchronous on its device's current stream.  Inference only (no autograd)."""
    from .propagation import propagate
    B = pred_init.shape[0]
    devs = [torch.device(d) for d in devices]
    if not devs:
        raise ValueError("propagate_sharded needs at least one device")
    home = pred_init.device
    parts = []
    with torch.no_grad():
        for r, d in enumerate(devs):
            lo, hi = shard_range(B, len(devs), r)
            if lo == hi:
                continue
            mv = lambda t: None if t is None else t[lo:hi].to(d, non_blocking=True)  # noqa: E731
            with torch.cuda.device(d):
                parts.append(propagate(mv(pred_init), mv(dep), mv(confidence), mv(aff), mv(offset),
                                       gamma.detach().to(d), **kw))
    out = {}
    for key in ("pred", "offset", "aff", "confidence"):
        vals = [p[key] for p in parts]
        out[key] = None if vals[0] is None else torch.cat([v.to(home) for v in vals], 0)
    inter = torch.cat([p["pred_inter_tensor"].to(home) for p in parts], 1)
    out["pred_inter"] = list(inter.unbind(0))
    out["pred_inter_tensor"] = inter
    return out


def devices_available(n: Optional[int] = None) -> list:
    """cuda:0 .. cuda:n-1 (all visible GPUs when n is None)."""
    count = torch.cuda.device_count()
    n = count if n is None else min(n, count)
    return [torch.device("cuda", i) for i in range(n)]
