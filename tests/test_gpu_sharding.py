"""GPU: the DataParallel-style batch scatter of the propagation section (verdict r2
item 6).  The reference runs its model under nn.DataParallel (src/main.py:366): dim-0
chunks of the batch on each device, outputs gathered back.  sharding.propagate_sharded
does the same for the section; each image's T iterations depend only on that image, so
the gathered result must equal the whole-batch section bit for bit — also when the
shards take a different kernel path than the whole batch (C3 whole: two resident image
groups in one launch; a shard of 2 KITTI images: one group).  With one GPU on the box
the shards go to the same device (the code path is the multi-device one: per-shard
device guard, copies, gather)."""
import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import propagate
from nlspn_eccv20_amd.sharding import devices_available, propagate_sharded, shard_range
from nlspn_eccv20_amd.synthetic import synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _inputs(B, H, W, density):
    s = synth(B, H, W, 8, seed=7240, density=density)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(DEV)  # noqa: E731
    oa = t(s["off_aff"])
    return t(s["pred_init"]), t(s["dep"]), t(s["conf"]), oa[:, 16:], oa[:, :16], torch.tensor([4.0], device=DEV)


@pytest.mark.parametrize("B,H,W,ndev,density", [
    (4, 240, 1216, 2, 0.05),   # C3 over two shards (the C4 per-rank shape at half the batch)
    (5, 228, 304, 2, 0.0072),  # uneven chunks (3 + 2), NYU
    (3, 64, 96, 4, 0.05),      # more devices than images: a trailing device gets nothing
])
def test_propagate_sharded_bitexact(B, H, W, ndev, density):
    pi, dep, conf, aff, off, g = _inputs(B, H, W, density)
    with torch.no_grad():
        whole = propagate(pi, dep, conf, aff, off, g, prop_time=18)
        sh = propagate_sharded(pi, dep, conf, aff, off, g, devices=[DEV] * ndev, prop_time=18)
    torch.cuda.synchronize()
    for k in ("pred", "pred_inter_tensor", "aff", "offset", "confidence"):
        assert torch.equal(sh[k], whole[k]), k
    assert len(sh["pred_inter"]) == 18
    sizes = [shard_range(B, ndev, r) for r in range(ndev)]
    assert sizes[0][0] == 0 and sizes[-1][1] == B


def test_propagate_sharded_over_visible_devices():
    """Every visible GPU (one on the test box, eight on a full node)."""
    devs = devices_available()
    pi, dep, conf, aff, off, g = _inputs(len(devs) * 2, 48, 64, 0.05)
    with torch.no_grad():
        whole = propagate(pi, dep, conf, aff, off, g, prop_time=6)
        sh = propagate_sharded(pi, dep, conf, aff, off, g, devices=devs, prop_time=6)
    torch.cuda.synchronize()
    assert torch.equal(sh["pred"], whole["pred"]) and torch.equal(sh["pred_inter_tensor"], whole["pred_inter_tensor"])
