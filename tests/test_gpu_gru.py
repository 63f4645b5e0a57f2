"""GPU: the GRU-mode convolutions on the HIP kernels (nlspn_eccv20_amd/gru.py,
csrc/nlspn_gconv.h) against the torch modules they replace (nlspnmodel.py:122-143,
365-373, 386-403), and the whole GRU-mode section against the module path.

Bar: f32 products and f32 accumulation on both sides, only the summation order differs —
relative L2 <= 1e-5 per layer (K up to 2304 terms), and the reference's own GRU-mode
fixtures at their 1e-4 RMSE bar (tests/test_backward_golden.py::test_gru_offset_matches_reference
runs the native path when gradients are off)."""
import types

import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import NLSPNModel
from nlspn_eccv20_amd.gru import GruConvs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model(H, W, seed=0, hc=128, K=8):
    args = types.SimpleNamespace(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=6,
                                 preserve_input=True, always_clip=False, conf_prop=True, offset=True,
                                 network="resnet34", from_scratch=True, zero_init_aff=False, use_GRU=True,
                                 use_S2D=False, GRU_hidden_dim=hc, GRU_input_dim=hc, lr=1e-3, max_depth=10.0,
                                 patch_height=H, patch_width=W, model_name="NLSPN")
    torch.manual_seed(seed)
    m = NLSPNModel(args).to(DEV).eval()
    # non-trivial biases and weights of a trained scale (the reference's init leaves small ones)
    with torch.no_grad():
        for mod in (m.encode_dep, m.encode_aff, m.GRU, m.decode_aff):
            for p in mod.parameters():
                p.add_(0.02 * torch.randn_like(p))
    return m


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.parametrize("B,H,W", [(8, 228, 304), (2, 240, 1216), (1, 50, 70)])
def test_gru_mode_convs_match_modules(B, H, W):
    m = _model(H, W)
    gc = GruConvs()
    assert GruConvs.supported(m)
    P = gc.pack(m)
    g = torch.Generator(device=DEV).manual_seed(3)
    new_pred = torch.rand((B, 1, H, W), device=DEV, generator=g) * 10
    aff = torch.rand((B, 9, H, W), device=DEV, generator=g)
    with torch.no_grad():
        d_ref = m.encode_dep(new_pred / m.args.max_depth)
        d = gc.encode_dep(P, new_pred, m.args.max_depth)
        assert d.shape == d_ref.shape
        assert _rel(d, d_ref) <= 1e-5, _rel(d, d_ref)
        a_ref = m.encode_aff(aff)
        a = gc.encode_aff(P, aff)
        assert _rel(a, a_ref) <= 1e-5, _rel(a, a_ref)
        h_ref = m.GRU(h=a_ref, x=d_ref)
        h = gc.gru(P, a_ref, d_ref)
        assert _rel(h, h_ref) <= 1e-5, _rel(h, h_ref)
        o_ref = m.decode_aff(h_ref)[:, :, :H, :W]
        o = gc.decode_aff(P, h_ref, (H, W))
        assert o.shape == o_ref.shape
        assert _rel(o, o_ref) <= 1e-5, _rel(o, o_ref)


def test_gru_mode_section_native_vs_modules():
    """The whole GRU-mode section (propagate_heads, inference) with the native convolutions
    against the torch-module path on the same model: every output within 1e-4 RMSE."""
    B, H, W = 2, 228, 304
    m = _model(H, W, seed=5)
    g = torch.Generator(device=DEV).manual_seed(9)
    pred_init = torch.rand((B, 1, H, W), device=DEV, generator=g) * 10
    dep = pred_init * (torch.rand((B, 1, H, W), device=DEV, generator=g) < 0.01)
    off_aff = torch.randn((B, 24, H, W), device=DEV, generator=g)
    conf = torch.rand((B, 1, H, W), device=DEV, generator=g)
    with torch.no_grad():
        o = m.propagate_heads(pred_init, off_aff, conf, dep)
        m.native_gru = False
        r = m.propagate_heads(pred_init, off_aff, conf, dep)
        m.native_gru = True
    for k in ("pred", "aff"):
        e = float(torch.sqrt(torch.mean((o[k].double() - r[k].double()) ** 2)))
        assert e <= 1e-4, (k, e)
    for a, b in zip(o["pred_inter"], r["pred_inter"]):
        assert float(torch.sqrt(torch.mean((a.double() - b.double()) ** 2))) <= 1e-4
    assert np.isfinite(o["pred"].cpu().numpy()).all()


@pytest.mark.parametrize("kind", ["AS", "ASS", "TC", "TGASS"])
@pytest.mark.parametrize("B,H,W", [(8, 228, 304), (1, 50, 70), (2, 17, 33)])
def test_decode_aff_fused_normalisation_bitequal(kind, B, H, W):
    """nlspn_gconv_affnorm (decode_aff's last transposed conv with the affinity normalisation
    and the reference-tap insert in its epilogue, nlspnmodel.py:179-201, :261-269) against the
    same conv storing the raw taps followed by nlspn_affinity_normalize: bit-equal, every plane,
    crop included; and the raw taps' normalisation within the kernels' own check of the tap sum."""
    from nlspn_eccv20_amd.propagation import affinity_normalization
    m = _model(H, W, seed=11)
    gc = GruConvs()
    P = gc.pack(m)
    g = torch.Generator(device=DEV).manual_seed(4)
    h = torch.randn((B, 128, (H + 7) // 8, (W + 7) // 8), device=DEV, generator=g)
    gamma = torch.tensor([0.37], device=DEV)
    with torch.no_grad():
        raw = gc.decode_aff(P, h, (H, W))
        ref = affinity_normalization(raw, gamma, kind)
        fused = gc.decode_aff(P, h, (H, W), gamma=gamma, kind=kind)
    assert fused.shape == (B, 9, H, W) == ref.shape
    assert torch.equal(fused, ref), float((fused - ref).abs().max())
    assert torch.allclose(fused.sum(1), torch.ones((B, H, W), device=DEV), atol=1e-5)
