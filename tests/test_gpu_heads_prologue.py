"""GPU: the head epilogue with the propagation prologue fused in
(nlspn_head_epilogue_prologue) + the loop from the prologued planes
(nlspn_propagate_normalized) give the same bits as the unfused path — the raw head
epilogue, then nlspn_propagate (whose step 1 runs _off_insert, the affinity
normalisation and the blends, nlspnmodel.py:323-348) — for every affinity kind and
flag set, on the resident and the per-iteration paths.  The convolution sums are the
same kernel's in both, so every output-dict tensor must be bit-identical."""
import pytest
import torch
import torch.nn as nn

from nlspn_eccv20_amd import propagate, propagate_normalized
from nlspn_eccv20_amd.heads import HeadWeights, head_epilogue, head_epilogue_prologue

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(B, C, H, W, seed=0, with_cf=True, depth_scale=10.0):
    torch.manual_seed(seed)
    oa = nn.Conv2d(2 * C, 24, 3, padding=1).to(DEV)
    idc = nn.Conv2d(2 * C, 1, 3, padding=1).to(DEV)
    cfc = nn.Conv2d(2 * C, 1, 3, padding=1).to(DEV) if with_cf else None
    with torch.no_grad():
        oa.weight.mul_(3.0)  # offsets of a few pixels, affinities of either sign
        idc.bias.add_(2.0)
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    src = [torch.rand((B, C, H, W), device=DEV, generator=g) for _ in range(4)]
    dep = torch.rand((B, 1, H, W), device=DEV, generator=g) * depth_scale
    dep = dep * (torch.rand((B, 1, H, W), device=DEV, generator=g) < 0.05)
    return oa, idc, cfc, src, dep


def _run_both(oa, idc, cfc, src, dep, gamma, kind, T, preserve, clip):
    fe1, fd_oa, fd_id, fd_cf = src
    hw = HeadWeights()
    with torch.no_grad():
        pi, off_aff, conf = head_epilogue(fe1, fd_oa, oa, fd_id, idc, fd_cf if cfc else None, cfc, weights=hw)
        ref = propagate(pi, dep if preserve else None, conf, off_aff[:, 16:], off_aff[:, :16], gamma, prop_time=T,
                        affinity=kind, preserve_input=preserve, always_clip=clip)
        h = head_epilogue_prologue(fe1, fd_oa, oa, fd_id, idc, dep if preserve else None, gamma, kind,
                                   fd_cf if cfc else None, cfc, preserve, clip, weights=hw)
        o = propagate_normalized(h["p0"], dep if preserve else None, h["confidence"], h["aff"], h["offset"], T,
                                 3, preserve, clip)
    torch.cuda.synchronize()
    return pi, ref, h, o


def _assert_same(pi, ref, h, o, with_cf):
    assert torch.equal(h["pred_init"], pi)
    assert torch.equal(h["aff"], ref["aff"])
    assert torch.equal(h["offset"], ref["offset"])
    if with_cf:
        assert torch.equal(h["confidence"], ref["confidence"])
    else:
        assert h["confidence"] is None
    assert torch.equal(o["pred_inter_tensor"], ref["pred_inter_tensor"])
    assert torch.equal(o["pred"], ref["pred"])


@pytest.mark.parametrize("kind", ["TGASS", "AS", "ASS", "TC"])
@pytest.mark.parametrize("preserve,clip", [(True, False), (False, True), (True, True)])
def test_fused_prologue_bitexact(kind, preserve, clip):
    oa, idc, cfc, src, dep = _case(2, 64, 40, 64, seed=1)
    gamma = torch.tensor([4.0], device=DEV)
    _assert_same(*_run_both(oa, idc, cfc, src, dep, gamma, kind, 18, preserve, clip), True)


@pytest.mark.parametrize("B,C,H,W,T,with_cf", [
    (2, 64, 228, 304, 18, True),   # NYU size: the resident path
    (3, 32, 37, 50, 6, True),      # W % 4 != 0: scalar kernels, per-iteration steps, partial tiles
    (1, 16, 24, 32, 1, False),     # T = 1, no confidence head
    (2, 16, 24, 32, 2, True),      # T = 2
])
def test_fused_prologue_shapes(B, C, H, W, T, with_cf):
    oa, idc, cfc, src, dep = _case(B, C, H, W, seed=2, with_cf=with_cf)
    gamma = torch.tensor([4.0], device=DEV)
    _assert_same(*_run_both(oa, idc, cfc, src, dep, gamma, "TGASS", T, True, False), with_cf)


def test_fused_prologue_per_iteration_path(monkeypatch):
    """propagate_normalized's per-iteration fallback (NLSPN_RESIDENT=0) at a width the
    resident kernel would take: the same bits as the unfused path."""
    monkeypatch.setenv("NLSPN_RESIDENT", "0")
    oa, idc, cfc, src, dep = _case(2, 16, 40, 64, seed=4)
    gamma = torch.tensor([4.0], device=DEV)
    _assert_same(*_run_both(oa, idc, cfc, src, dep, gamma, "TGASS", 7, True, False), True)


def test_fused_prologue_negative_depth_clip():
    """always_clip with heads that predict negative depth (clamp in p0 and every step)."""
    oa, idc, cfc, src, dep = _case(2, 16, 24, 64, seed=3)
    with torch.no_grad():
        idc.bias.sub_(6.0)
    gamma = torch.tensor([2.5], device=DEV)
    _assert_same(*_run_both(oa, idc, cfc, src, dep, gamma, "TGASS", 5, True, True), True)


def test_model_forward_fused_equals_unfused():
    """NLSPNModel.forward at inference takes the fused path (3x3, K=8, offsets, no GRU)
    and returns the output dict of heads() + propagate_heads() bit for bit."""
    import types
    from nlspn_eccv20_amd import NLSPNModel
    args = types.SimpleNamespace(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=18,
                                 preserve_input=True, always_clip=False, conf_prop=True, offset=True,
                                 network="resnet18", from_scratch=True, zero_init_aff=False, use_GRU=False,
                                 use_S2D=False, GRU_hidden_dim=8, GRU_input_dim=8, lr=1e-3, max_depth=10.0,
                                 patch_height=48, patch_width=80, model_name="NLSPN")
    torch.manual_seed(0)
    m = NLSPNModel(args).to(DEV).eval()
    g = torch.Generator(device=DEV).manual_seed(5)
    rgb = torch.rand((2, 3, 48, 80), device=DEV, generator=g)
    dep = torch.rand((2, 1, 48, 80), device=DEV, generator=g) * 10 * (torch.rand((2, 1, 48, 80), device=DEV,
                                                                                   generator=g) < 0.05)
    s = {"rgb": rgb, "dep": dep}
    with torch.no_grad():
        # one decoder pass for both (MIOpen may pick another algorithm on a second pass)
        fe1, id_fd1, oa_fd1, cf_fd1 = m._decoder(s)
        fused = m._forward_fused(fe1, id_fd1, oa_fd1, cf_fd1, dep)
        ref = m.propagate_heads(*head_epilogue(fe1, oa_fd1, m.off_aff_dec0, id_fd1, m.id_dec0, cf_fd1, m.cf_dec0,
                                               weights=m._head_weights), dep)
        whole = m(s)  # forward() takes the fused path
    for k in ("pred", "pred_init", "offset", "aff", "confidence"):
        assert torch.equal(fused[k], ref[k]), k
    assert all(torch.equal(a, b) for a, b in zip(fused["pred_inter"], ref["pred_inter"]))
    for k in ("pred", "aff", "offset"):  # up to the decoder's run-to-run rounding
        assert torch.allclose(whole[k], ref[k], rtol=1e-4, atol=1e-4), k


def test_model_forward_fused_coerces_dep():
    """The fused inference path accepts the depth batches the unfused path does (ADVICE
    r2): a non-contiguous or float64 dep gives the float32-contiguous result."""
    import types
    from nlspn_eccv20_amd import NLSPNModel
    args = types.SimpleNamespace(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=6,
                                 preserve_input=True, always_clip=False, conf_prop=True, offset=True,
                                 network="resnet18", from_scratch=True, zero_init_aff=False, use_GRU=False,
                                 use_S2D=False, GRU_hidden_dim=8, GRU_input_dim=8, lr=1e-3, max_depth=10.0,
                                 patch_height=48, patch_width=80, model_name="NLSPN")
    torch.manual_seed(0)
    m = NLSPNModel(args).to(DEV).eval()
    g = torch.Generator(device=DEV).manual_seed(6)
    rgb = torch.rand((2, 3, 48, 80), device=DEV, generator=g)
    dep = torch.rand((2, 1, 48, 80), device=DEV, generator=g) * 10 * (torch.rand((2, 1, 48, 80), device=DEV,
                                                                                   generator=g) < 0.05)
    wide = torch.zeros((2, 1, 48, 160), device=DEV)
    wide[..., ::2] = dep
    with torch.no_grad():
        fe1, id_fd1, oa_fd1, cf_fd1 = m._decoder({"rgb": rgb, "dep": dep})
        ref = m._forward_fused(fe1, id_fd1, oa_fd1, cf_fd1, dep)
        strided = m._forward_fused(fe1, id_fd1, oa_fd1, cf_fd1, wide[..., ::2])
        f64 = m._forward_fused(fe1, id_fd1, oa_fd1, cf_fd1, dep.double())
    for o in (strided, f64):
        for k in ("pred", "aff", "confidence"):
            assert torch.equal(o[k], ref[k]), k


def test_replica_does_not_use_the_head_cache():
    """DataParallel replicas share the module's __dict__ (so its packed-weight cache) but
    hold fresh parameter copies: they pack per call."""
    import types
    from nlspn_eccv20_amd import NLSPNModel
    args = types.SimpleNamespace(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=6,
                                 preserve_input=True, always_clip=False, conf_prop=True, offset=True,
                                 network="resnet18", from_scratch=True, zero_init_aff=False, use_GRU=False,
                                 use_S2D=False, GRU_hidden_dim=8, GRU_input_dim=8, lr=1e-3, max_depth=10.0,
                                 patch_height=48, patch_width=80, model_name="NLSPN")
    m = NLSPNModel(args).to(DEV).eval()
    assert m._head_cache() is m._head_weights
    rep = torch.nn.parallel.replicate(m, [0], detach=True)[0]
    assert getattr(rep, "_is_replica", False) and rep._head_cache() is None
