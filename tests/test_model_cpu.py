"""The drop-in NLSPNModel (nlspn_eccv20_amd/model.py) on the CPU: module tree and
state_dict compatibility with the reference, head shapes, registry, pretrained
load.  The propagation section itself needs the GPU (tests/test_gpu_model.py).

state_dict_keys.json is generated from the reference's own NLSPNModel.__init__
(tests/golden/gen_golden.py, section 6) with the torchvision ResNet stages
stubbed empty; the stage keys (conv2/conv3/conv4) are checked against
torchvision's BasicBlock naming instead (resnet34 = 3/4/6 blocks)."""
import json
import os
import types

import pytest
import torch

from nlspn_eccv20_amd import NLSPNModel
from nlspn_eccv20_amd import model as M

from conftest import GOLDEN_DIR


def make_args(**kw):
    a = dict(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=18, preserve_input=True,
             always_clip=False, conf_prop=True, offset=True, network="resnet34", from_scratch=True,
             zero_init_aff=True, use_GRU=True, use_S2D=True, GRU_hidden_dim=128, GRU_input_dim=128, lr=1e-3,
             max_depth=10.0, patch_height=64, patch_width=96, model_name="NLSPN")
    a.update(kw)
    return types.SimpleNamespace(**a)


def stage_keys(blocks):
    """torchvision resnet layer1..layer3 state_dict keys -> shapes (BasicBlock)."""
    out = {}
    inpl = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256), blocks)):
        stage = f"conv{li + 2}"
        for b in range(n):
            cin = inpl if b == 0 else planes
            pre = f"{stage}.{b}."
            out[pre + "conv1.weight"] = [planes, cin, 3, 3]
            out[pre + "conv2.weight"] = [planes, planes, 3, 3]
            for bn in ("bn1", "bn2"):
                for s in ("weight", "bias", "running_mean", "running_var"):
                    out[f"{pre}{bn}.{s}"] = [planes]
                out[f"{pre}{bn}.num_batches_tracked"] = []
            if b == 0 and li > 0:
                out[pre + "downsample.0.weight"] = [planes, cin, 1, 1]
                for s in ("weight", "bias", "running_mean", "running_var"):
                    out[f"{pre}downsample.1.{s}"] = [planes]
                out[pre + "downsample.1.num_batches_tracked"] = []
        inpl = planes
    return out


@pytest.mark.parametrize("tag,kw", [
    ("gru_s2d_offset", dict()),
    ("plain", dict(offset=False, use_GRU=False, use_S2D=False)),
])
def test_state_dict_matches_reference(tag, kw):
    ref = json.load(open(os.path.join(GOLDEN_DIR, "state_dict_keys.json")))[tag]
    ref.update(stage_keys((3, 4, 6)))
    m = NLSPNModel(make_args(**kw))
    got = {k: list(v.shape) for k, v in m.state_dict().items()}
    assert got == ref
    # the reference's parameter-group order (nlspnmodel.py:158-159): trainable params only
    assert len(m.param_groups[0]["params"]) == sum(1 for p in m.parameters() if p.requires_grad)


def test_resnet18_stages():
    m = NLSPNModel(make_args(network="resnet18", use_GRU=False))
    keys = {k: list(v.shape) for k, v in m.state_dict().items() if k.split(".")[0] in ("conv2", "conv3", "conv4")}
    assert keys == stage_keys((2, 2, 2))


def test_reference_checkpoint_loads():
    """A state_dict with the reference's keys loads strictly (resume / pretrained eval)."""
    a = NLSPNModel(make_args())
    b = NLSPNModel(make_args())
    b.load_state_dict(a.state_dict(), strict=True)
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_pretrained_resnet_loads_weights_only(tmp_path, monkeypatch):
    """get_resnet34(pretrained=True) reads pretrained/resnet34.pth (common.py:27-42) with a
    loader that executes nothing (weights_only=True) and keeps layer1..layer3."""
    src = M._ResNetStages((3, 4, 6))
    sd = {k: v.clone() for k, v in src.state_dict().items()}
    sd["fc.weight"] = torch.zeros(10, 512)  # torchvision checkpoints carry more keys
    os.makedirs(tmp_path / "pretrained")
    torch.save(sd, tmp_path / "pretrained" / "resnet34.pth")
    monkeypatch.chdir(tmp_path)
    m = NLSPNModel(make_args(from_scratch=False))
    assert torch.equal(m.conv3[0].conv1.weight, src.layer2[0].conv1.weight)


@pytest.mark.parametrize("kw", [dict(), dict(offset=False, conf_prop=False, use_S2D=False)])
def test_heads_shapes(kw):
    torch.manual_seed(0)
    m = NLSPNModel(make_args(**kw)).eval()
    B, H, W = 1, 60, 84  # not multiples of 8: decoder crops (_concat, nlspnmodel.py:161-177)
    dep = torch.rand(B, 1, H, W) * (torch.rand(B, 1, H, W) < 0.05)
    with torch.no_grad():
        pi, oa, cf = m.heads({"rgb": torch.rand(B, 3, H, W), "dep": dep})
    K = 8
    assert pi.shape == (B, 1, H, W)
    assert oa.shape == (B, 3 * K if m.args.offset else K, H, W)
    assert (cf is None) == (not m.args.conf_prop)
    if cf is not None:
        assert cf.shape == (B, 1, H, W) and (cf >= 0).all() and (cf <= 1).all()


def test_s2d_min_pool():
    """S2D's min-pool treats zeros as missing (nlspnmodel.py:437-447)."""
    s = M.S2D()
    dep = torch.zeros(1, 1, 9, 9)
    dep[0, 0, 4, 4] = 3.0
    dep[0, 0, 4, 5] = 5.0
    z = -s.min_pools[0](torch.where(dep == 0, -999 * torch.ones_like(dep), -dep))
    z = torch.where(z == 999, torch.zeros_like(dep), z)
    assert z[0, 0, 4, 4] == 3.0 and z[0, 0, 4, 6] == 5.0 and z[0, 0, 0, 0] == 0.0


def test_registry():
    assert M.get(make_args()) is NLSPNModel
    with pytest.raises(NotImplementedError):
        M.get(make_args(model_name="Other"))


def test_dataparallel_wraps_model():
    """The reference wraps the model in nn.DataParallel (src/main.py:366); the drop-in
    must construct under it with the same state_dict (module.-prefixed) and expose the
    propagation module.  (Multi-GPU scatter itself: sharding.propagate_sharded / bench.)"""
    m = NLSPNModel(make_args())
    dp = torch.nn.DataParallel(m)
    keys = set(dp.state_dict())
    assert keys == {"module." + k for k in m.state_dict()}
    dp2 = torch.nn.DataParallel(NLSPNModel(make_args()))
    dp2.load_state_dict(dp.state_dict(), strict=True)
    assert dp.module is m
