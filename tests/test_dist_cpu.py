"""World-size-2 gloo test of the multi-GPU path's logic on CPU: batch shards are
processed independently (no data-path collective) and reassemble to exactly the
single-process result; the timing reduction takes the max over ranks."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from nlspn_eccv20_amd.sharding import max_over_ranks, shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from nlspn_eccv20_amd.synthetic import synth
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = synth(5, 20, 28, 8, seed=77)
    lo, hi = shard_range(5, world, rank)
    sl = lambda x: x[lo:hi]  # noqa: E731
    o = O.propagate(sl(s["pred_init"]), sl(s["dep"]), sl(s["conf"]), sl(s["off_aff"])[:, 16:],
                    sl(s["off_aff"])[:, :16], 4.0)
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, o["pred"]))  # test-side gather only
    t = max_over_ranks(float(rank + 1))
    if rank == 0:
        full = O.propagate(s["pred_init"], s["dep"], s["conf"], s["off_aff"][:, 16:], s["off_aff"][:, :16], 4.0)
        got = np.concatenate([p[2] for p in sorted(parts, key=lambda p: p[0])], 0)
        q.put((bool(np.array_equal(got, full["pred"])), t))
    dist.destroy_process_group()


def test_shard_range():
    assert [shard_range(32, 8, r) for r in range(8)] == [(4 * r, 4 * r + 4) for r in range(8)]
    assert [shard_range(5, 2, r) for r in range(2)] == [(0, 3), (3, 5)]
    assert shard_range(2, 4, 3) == (2, 2)
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_gloo_two_ranks_shards_reassemble():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    equal, tmax = q.get(timeout=5)
    assert equal
    assert tmax == 2.0


def test_bench_launcher_spawns_ranks_dry_run():
    """bench.py --gpus 2 with no torchrun environment spawns 2 ranks itself
    (launch.spawn_local); --dry-run runs the launcher + sharding path on CPU (gloo):
    n_gpus = 2 and each rank owns its contiguous shard of the 2x global batch
    (C4's form: KITTI B=4 per GPU)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                          "--config", "kitti"], capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["global_batch"] == 8
    assert line["shards"] == [[0, 0, 4], [1, 4, 8]]


def test_spawn_local_propagates_failure():
    import sys
    from nlspn_eccv20_amd.launch import spawn_local
    code = "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"
    assert spawn_local(2, [sys.executable, "-c", code], timeout=60) == 3
    assert spawn_local(2, [sys.executable, "-c", "import os; assert os.environ['WORLD_SIZE'] == '2'"],
                       timeout=60) == 0
