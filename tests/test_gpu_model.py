"""The drop-in NLSPNModel on the GPU: heads on MIOpen, propagation on the HIP
kernels.  The propagation section is checked against the oracle on the model's
own head outputs; GRU mode against a restatement of nlspnmodel.py:335-373 that
runs every propagation step and affinity normalisation in the oracle and only the
GRU/encoder convolutions in torch.

Tolerances: fused section vs oracle f32: max |diff| <= 1e-4 (bit-exact kernels,
inputs identical); GRU mode: relative L2 <= 1e-4 (the GRU's MIOpen convolutions are
re-run on the oracle's iterates, so last-bit differences in either would show)."""
import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import NLSPNModel

from test_model_cpu import make_args

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def sample(B, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    dep = torch.rand(B, 1, H, W, generator=g) * 10 * (torch.rand(B, 1, H, W, generator=g) < 0.05)
    return {"rgb": torch.rand(B, 3, H, W, generator=g).to(DEV), "dep": dep.to(DEV)}


def randomize_aff_head(m, seed=1):
    """zero_init_aff makes every offset/affinity 0; give the heads random weights so
    the propagation sees non-trivial inputs."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.off_aff_dec0.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.05)
        if hasattr(m, "decode_aff"):
            for p in m.decode_aff[-1].parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)


np32 = lambda t: None if t is None else t.detach().float().cpu().numpy()  # noqa: E731


@pytest.mark.parametrize("kw", [
    dict(),
    dict(offset=False),
    dict(conf_prop=False),
    dict(always_clip=True, affinity="ASS"),
    dict(preserve_input=False),
])
def test_model_propagation_vs_oracle(oracle, kw):
    torch.manual_seed(0)
    m = NLSPNModel(make_args(use_GRU=False, prop_time=8, **kw)).to(DEV).eval()
    randomize_aff_head(m)
    s = sample(2, 48, 80)
    with torch.no_grad():
        pi, oa, cf = m.heads(s)
        out = m.propagate_heads(pi, oa, cf, s["dep"])
        full = m(s)
    a = m.args
    K = 8
    oa_n = np32(oa)
    ref = oracle.propagate(np32(pi), np32(s["dep"]) if a.preserve_input else None, np32(cf),
                           oa_n[:, 2 * K:] if a.offset else oa_n, oa_n[:, :2 * K] if a.offset else None,
                           float(m.aff_scale_const.item()), kind=a.affinity, prop_time=a.prop_time,
                           preserve_input=a.preserve_input, always_clip=a.always_clip)
    assert np.abs(np32(out["pred"]) - ref["pred"]).max() <= 1e-4
    assert np.abs(np32(out["aff"]) - ref["aff"]).max() <= 1e-6
    for t in range(a.prop_time):
        assert np.abs(np32(out["pred_inter"][t]) - ref["pred_inter"][t]).max() <= 1e-4
    if a.offset:
        assert np.array_equal(np32(out["offset"]), ref["offset"])
    if a.conf_prop:
        assert np.array_equal(np32(out["confidence"]), ref["confidence"])
    assert set(out) == {"pred", "pred_init", "pred_inter", "offset", "aff", "gamma", "confidence"}
    # forward() == heads() + propagate_heads(); MIOpen may pick another conv algorithm on
    # the second call, so the heads agree to rounding only
    d = (full["pred"] - out["pred"]).norm() / out["pred"].norm()
    assert d.item() <= 1e-4


def ref_gru_loop(oracle, m, pi, oa, cf, dep):
    """nlspnmodel.py:323-381 with use_GRU: oracle for normalisation and every step,
    the model's torch modules for encode_dep / encode_aff / GRU / decode_aff."""
    a = m.args
    K = m.num_neighbors
    gamma = float(m.aff_scale_const.item())
    oa = np32(oa)
    off = oracle.off_insert(oa[:, :2 * K]) if a.offset else None
    aff = oracle.affinity_normalization(oa[:, 2 * K:] if a.offset else oa, a.affinity, gamma)
    dep = np32(dep)
    mask = (dep > 0).astype(np.float32)
    conf = np32(cf)
    if conf is not None and a.preserve_input:
        conf = (1 - mask) * conf + mask
    x = np32(pi)
    if a.preserve_input:
        x = (1 - mask) * x + mask * dep
    if a.always_clip:
        x = np.maximum(x, 0)
    inter = []
    to_dev = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(DEV)  # noqa: E731
    for k in range(1, a.prop_time + 1):
        f = x * conf if conf is not None else x
        if off is not None:
            x = oracle.mdcn_c1(f, off, aff)
        else:
            x = oracle.prop_noffset(f, aff)
        if a.preserve_input:
            x = (1 - mask) * x + mask * dep
        if a.always_clip:
            x = np.maximum(x, 0)
        inter.append(x)
        if k < a.prop_time:
            dep_feat = m.encode_dep(to_dev(x) / a.max_depth)
            if k == 1:
                h = m.encode_aff(to_dev(aff))
            h = m.GRU(h=h, x=dep_feat)
            raw = np32(m.decode_aff(h)[:, :, :a.patch_height, :a.patch_width])
            aff = oracle.affinity_normalization(raw, a.affinity, gamma)
    pred = x if a.always_clip else np.maximum(x, 0)
    return pred, inter, aff


@pytest.mark.parametrize("kw", [dict(), dict(offset=False, use_S2D=False), dict(always_clip=True)])
def test_model_gru_vs_oracle(oracle, kw):
    torch.manual_seed(0)
    H, W = 48, 80
    m = NLSPNModel(make_args(prop_time=6, patch_height=H, patch_width=W, **kw)).to(DEV).eval()
    randomize_aff_head(m)
    s = sample(2, H, W, seed=3)
    with torch.no_grad():
        pi, oa, cf = m.heads(s)
        out = m.propagate_heads(pi, oa, cf, s["dep"])
        pred, inter, aff = ref_gru_loop(oracle, m, pi, oa, cf, s["dep"])
    rel = lambda u, v: float(np.linalg.norm(u - v) / max(np.linalg.norm(v), 1e-30))  # noqa: E731
    assert rel(np32(out["pred"]), pred) <= 1e-4
    assert len(out["pred_inter"]) == m.args.prop_time
    assert rel(np32(out["pred_inter"][0]), inter[0]) <= 1e-6
    assert rel(np32(out["aff"]), aff) <= 1e-4


def test_model_gru_trains():
    """GRU mode with gradients: the differentiable path (torch prologue, step-level
    backward kernels) gives the same forward as the fused inference path, and its
    gradient agrees with a central finite difference of the loss along a random
    direction in the GRU / decode_aff weights (smooth in them: offsets are fixed)."""
    torch.manual_seed(0)
    H, W = 32, 48
    m = NLSPNModel(make_args(prop_time=4, patch_height=H, patch_width=W)).to(DEV).train()
    randomize_aff_head(m)
    for mod in m.modules():  # no batch statistics: forward must be a fixed function of the weights
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.eval()
    s = sample(2, H, W, seed=7)
    with torch.no_grad():
        ref = m(s)
    out = m(s)
    d = (out["pred"] - ref["pred"]).norm() / ref["pred"].norm()
    assert d.item() <= 1e-5
    gt = torch.rand(2, 1, H, W, device=DEV) * 10
    loss = ((out["pred"] - gt) ** 2).mean()
    loss.backward()
    params = [p for n, p in m.named_parameters() if n.startswith(("GRU.", "decode_aff.", "encode_aff."))]
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in params)
    assert sum(p.grad.abs().sum().item() for p in params) > 0
    g = torch.Generator(device=DEV).manual_seed(1)
    # direction scaled to each tensor's weight magnitude; eps = 1 % of it
    v = [torch.randn(p.shape, device=DEV, generator=g) * (p.detach().abs().mean() + 1e-3) for p in params]
    dd = sum((p.grad * u).sum().item() for p, u in zip(params, v))
    eps = 1e-2
    with torch.no_grad():
        def lossv(sign):
            for p, u in zip(params, v):
                p.add_(sign * eps * u)
            r = ((m(s)["pred"] - gt) ** 2).mean().item()
            for p, u in zip(params, v):
                p.sub_(sign * eps * u)
            return r
        fd = (lossv(1.0) - lossv(-1.0)) / (2 * eps)
    assert abs(fd - dd) <= 2e-2 * max(abs(dd), 1e-6), (fd, dd)


def test_model_trains_end_to_end():
    """Non-GRU model in training mode: loss.backward() reaches every head through the
    native propagation backward, and an optimizer step changes the weights."""
    torch.manual_seed(0)
    m = NLSPNModel(make_args(use_GRU=False, prop_time=6)).to(DEV).train()
    randomize_aff_head(m)
    opt = torch.optim.Adam(m.param_groups, lr=1e-3)
    s = sample(2, 48, 80, seed=5)
    gt = torch.rand(2, 1, 48, 80, device=DEV) * 10
    out = m(s)
    loss = ((out["pred"] - gt) ** 2).mean()
    loss.backward()
    for name in ("id_dec0.0.weight", "off_aff_dec0.0.weight", "cf_dec0.0.weight", "aff_scale_const",
                 "conv1_rgb.0.weight"):
        p = dict(m.named_parameters())[name]
        assert p.grad is not None and torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0, name
    w0 = m.off_aff_dec0[0].weight.detach().clone()
    opt.step()
    assert not torch.equal(w0, m.off_aff_dec0[0].weight)


def test_model_nyu_size_gru():
    """The reference's NYU configuration (228x304 patch, resnet34, GRU, S2D, offsets, T=18)."""
    torch.manual_seed(0)
    m = NLSPNModel(make_args(patch_height=228, patch_width=304)).to(DEV).eval()
    randomize_aff_head(m)
    s = sample(2, 228, 304)
    with torch.no_grad():
        out = m(s)
    assert out["pred"].shape == (2, 1, 228, 304) and torch.isfinite(out["pred"]).all()
    assert (out["pred"] >= 0).all() and len(out["pred_inter"]) == 18


@pytest.mark.parametrize("use_gru", [True, False])
def test_section_graph_equals_eager(use_gru):
    """SectionGraph (the section captured into one hipGraph, GRU convolutions included)
    replays exactly what the eager section computes, and picks up new head outputs."""
    from nlspn_eccv20_amd import SectionGraph
    torch.manual_seed(0)
    m = NLSPNModel(make_args(use_GRU=use_gru, prop_time=6, patch_height=48, patch_width=80)).to(DEV).eval()
    randomize_aff_head(m)
    s1, s2 = sample(2, 48, 80, seed=3), sample(2, 48, 80, seed=4)
    with torch.no_grad():
        h1, h2 = m.heads(s1), m.heads(s2)
        g = SectionGraph(m, *h1, s1["dep"])
        for h, smp in ((h1, s1), (h2, s2), (h1, s1)):
            eager = m.propagate_heads(*h, smp["dep"])
            o = g.replay(*h, smp["dep"])
            torch.cuda.synchronize()
            if use_gru:  # MIOpen may choose another conv algorithm per call: rounding-level only
                for a, b in zip(o["pred_inter"] + [o["pred"]], eager["pred_inter"] + [eager["pred"]]):
                    assert ((a - b).norm() / b.norm()).item() <= 1e-5
            else:
                assert torch.equal(o["pred"], eager["pred"])
                for a, b in zip(o["pred_inter"], eager["pred_inter"]):
                    assert torch.equal(a, b)


def test_gru_channels_last_equals_default():
    """gru_channels_last (the GRU-mode convolutions in NHWC) computes the same section:
    the same convolutions in another layout (MIOpen may pick another algorithm, so f32
    rounding differs; the propagated depth agrees to 1e-4 of its range)."""
    torch.manual_seed(0)
    m = NLSPNModel(make_args(prop_time=6, patch_height=48, patch_width=80)).to(DEV).eval()
    randomize_aff_head(m)
    s = sample(2, 48, 80, seed=5)
    with torch.no_grad():
        h = m.heads(s)
        ref = m.propagate_heads(*h, s["dep"])
        m.gru_channels_last()
        got = m.propagate_heads(*h, s["dep"])
    scale = ref["pred"].abs().max().item()
    assert (got["pred"] - ref["pred"]).abs().max().item() <= 1e-4 * scale
    assert (got["aff"] - ref["aff"]).abs().max().item() <= 1e-4
