"""One process per GPU on one node without an external launcher.

The reference scatters a batch over GPUs with nn.DataParallel (src/main.py:366) or
spawns one process per GPU (src/main.py:432-433).  Here `spawn_local` starts N
fresh copies of a command, one per GPU, with the torchrun environment (RANK,
LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT); the parent never
touches the GPU (it only waits), so no HIP state is inherited or exec'd over.
`init_from_env` is the worker side.  No collective runs on the data path: batch
shards are independent (sharding.shard_range); the process group carries only
timing reductions.
"""
from __future__ import annotations

import os
import socket
import subprocess
import time
from typing import Optional, Sequence

import torch
import torch.distributed as dist


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_local(nprocs: int, cmd: Sequence[str], env: Optional[dict] = None, timeout: Optional[float] = None) -> int:
    """Run `cmd` as `nprocs` ranks on this node; return the first non-zero exit code
    (0 when every rank succeeded).  A failing rank stops the others (exact PIDs)."""
    if nprocs < 1:
        raise ValueError(f"nprocs must be >= 1, got {nprocs}")
    port = free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(list(cmd), env=e))
    t0 = time.monotonic()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if timeout is not None and time.monotonic() - t0 > timeout and live:
            for q in live:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    return rc


def env_rank() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the torchrun-style environment (1, 0, 0 if unset)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_from_env(backend: str = "nccl") -> tuple[int, int, int]:
    """Join the process group described by the environment.  With `nccl` (RCCL on ROCm)
    the rank's device is cuda:LOCAL_RANK.  Returns (world, rank, local_rank)."""
    world, rank, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local
