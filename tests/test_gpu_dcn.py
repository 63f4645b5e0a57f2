"""GPU: seam 2 of the drop-in — the `DCN` module (vision.cpp:9-10) on MI355X:
generic modulated DCNv2 forward and backward against the oracle's restatement
(tests/test_oracle_dcn.py pins it), through the reference's own call shape
(ModulatedDeformConvFunction.apply, modulated_deform_conv_func.py:15-56).

Tolerances: float32 kernels vs the float64 oracle on the same float32 inputs —
relative L2 <= 1e-5 (forward) and <= 1e-4 (backward: grad_input is a float-atomic
scatter as in the reference, and the reference's columns come from BLAS in an
unspecified order, so no bit-exact claim is made for generic shapes).
"""
import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import dcn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CASES = [  # C, Cout, group, dg, kh, kw, stride, pad, dil
    (1, 1, 1, 1, 3, 3, (1, 1), (1, 1), (1, 1)),     # NLSPN's DCN call
    (4, 6, 2, 2, 3, 3, (1, 1), (1, 1), (1, 1)),     # groups + deformable groups
    (3, 5, 1, 3, 3, 3, (2, 2), (1, 1), (1, 1)),     # stride
    (2, 2, 1, 1, 3, 3, (1, 1), (2, 2), (2, 2)),     # dilation
    (1, 1, 1, 1, 1, 17, (1, 1), (0, 8), (1, 1)),    # NLSPN 1x17 geometry (pad_w != pad_h quirk)
    (8, 4, 4, 1, 5, 5, (1, 1), (2, 2), (1, 1)),
]


def _case(seed, C, Cout, group, dg, kh, kw, stride, pad, dil, B=2, H=13, W=17, sigma=2.0):
    rng = np.random.default_rng(seed)
    Ho = (H + 2 * pad[0] - (dil[0] * (kh - 1) + 1)) // stride[0] + 1
    Wo = (W + 2 * pad[1] - (dil[1] * (kw - 1) + 1)) // stride[1] + 1
    f32 = np.float32
    return (rng.standard_normal((B, C, H, W)).astype(f32), rng.standard_normal((Cout, C // group, kh, kw)).astype(f32),
            rng.standard_normal((Cout,)).astype(f32),
            (rng.standard_normal((B, 2 * dg * kh * kw, Ho, Wo)) * sigma).astype(f32),
            rng.random((B, dg * kh * kw, Ho, Wo)).astype(f32))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(DEV)  # noqa: E731


@pytest.mark.parametrize("case", CASES)
def test_dcn_forward_vs_oracle(oracle, case):
    C, Cout, group, dg, kh, kw, stride, pad, dil = case
    inp, wt, bias, off, mask = _case(1, *case)
    out = dcn.modulated_deform_conv_forward(cu(inp), cu(wt), cu(bias), cu(off), cu(mask), kh, kw, *stride, *pad,
                                            *dil, group, dg, 64)
    exp = oracle.mdcn_forward(*(x.astype(np.float64) for x in (inp, wt, bias, off, mask)), stride, pad, dil, group, dg)
    assert rel(out.cpu().numpy(), exp) <= 1e-5


@pytest.mark.parametrize("case", CASES)
def test_dcn_backward_vs_oracle(oracle, case):
    C, Cout, group, dg, kh, kw, stride, pad, dil = case
    inp, wt, bias, off, mask = _case(2, *case)
    x = [cu(a).requires_grad_(True) for a in (inp, off, mask, wt, bias)]
    out = dcn.ModulatedDeformConvFunction.apply(x[0], x[1], x[2], x[3], x[4], stride, pad, dil, group, dg, 64)
    go = torch.randn_like(out)
    out.backward(go)
    exp = oracle.mdcn_backward(*(a.astype(np.float64) for a in (inp, wt, off, mask)), go.cpu().double().numpy(),
                               stride, pad, dil, group, dg)
    gi, goff, gm, gw, gb = exp
    for name, got, want in (("input", x[0].grad, gi), ("offset", x[1].grad, goff), ("mask", x[2].grad, gm),
                            ("weight", x[3].grad, gw), ("bias", x[4].grad, gb)):
        assert rel(got.cpu().numpy(), want) <= 1e-4, name


def test_dcn_shim_runs_nlspn_step(oracle):
    """The reference's _propagate_once offset branch (nlspnmodel.py:204-208) through
    the DCN shim equals the fused prop_step (and the oracle) on the same inputs."""
    from nlspn_eccv20_amd import prop_step
    rng = np.random.default_rng(5)
    B, H, W = 2, 20, 24
    f = rng.random((B, 1, H, W)).astype(np.float32)
    off = (rng.standard_normal((B, 18, H, W)) * 2).astype(np.float32)
    off[:, 8:10] = 0  # reference tap: zero offset (_off_insert)
    aff = rng.random((B, 9, H, W)).astype(np.float32)
    aff[:, 4] = 1 - aff[:, [0, 1, 2, 3, 5, 6, 7, 8]].sum(1)
    w = torch.ones((1, 1, 3, 3), device=DEV)
    b = torch.zeros((1,), device=DEV)
    out = dcn.ModulatedDeformConvFunction.apply(cu(f), cu(off), cu(aff), w, b, 1, 1, 1, 1, 1, 64)
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.mdcn_c1(f, off, aff))
    fused = prop_step(cu(f), None, None, cu(aff), cu(off), preserve_input=False)
    np.testing.assert_allclose(out.cpu().numpy(), fused.cpu().numpy(), rtol=0, atol=2e-6)


def test_dcn_backward_errors():
    x = torch.zeros(1, 3, 8, 8, device=DEV)
    w = torch.zeros(4, 3, 3, 3, device=DEV)
    with pytest.raises(RuntimeError, match="must divide group"):
        dcn.modulated_deform_conv_backward(x, w, None, torch.zeros(1, 18, 8, 8, device=DEV),
                                           torch.zeros(1, 9, 8, 8, device=DEV), torch.zeros(1, 4, 8, 8, device=DEV),
                                           3, 3, 1, 1, 1, 1, 1, 1, 2, 1, 64)


# ------------------------------------------------------------------ float64 (seam 2)
# The reference dispatches float and double (AT_DISPATCH_FLOATING_TYPES, .cu:93 / .cu:221);
# the float64 kernels do double arithmetic throughout, so they meet the fp64 oracle to
# ~1e-12 relative (forward) — the only differences are summation order — and the
# reference-style gradcheck (deformconv/test.py:405-434, run here in float64 as
# torch.autograd.gradcheck expects) passes through ModulatedDeformConvFunction.
@pytest.mark.parametrize("case", CASES)
def test_dcn_float64_vs_oracle(oracle, case):
    C, Cout, group, dg, kh, kw, stride, pad, dil = case
    args64 = [x.astype(np.float64) for x in _case(3, *case)]
    inp, wt, bias, off, mask = (cu(x) for x in args64)
    out = dcn.modulated_deform_conv_forward(inp, wt, bias, off, mask, kh, kw, *stride, *pad, *dil, group, dg, 64)
    assert out.dtype == torch.float64
    exp = oracle.mdcn_forward(*args64, stride, pad, dil, group, dg)
    assert rel(out.cpu().numpy(), exp) <= 1e-12
    g = np.random.default_rng(4).standard_normal(out.shape)
    got = dcn.modulated_deform_conv_backward(inp, wt, bias, off, mask, cu(g), kh, kw, *stride, *pad, *dil, group,
                                             dg, 64)
    ref = oracle.mdcn_backward(args64[0], args64[1], args64[3], args64[4], g, stride, pad, dil, group, dg)
    for gt, rt in zip(got, ref):
        assert gt.dtype == torch.float64 and rel(gt.cpu().numpy(), rt) <= 1e-10


def test_dcn_gradcheck_float64():
    """torch.autograd.gradcheck of ModulatedDeformConvFunction in float64, the reference's
    check_gradient_mdconv setup (test.py:15-18, 405-434: N=2, inC=4, 4x4, outC=4, 3x3,
    groups 2, stride 1, padding 1)."""
    torch.manual_seed(0)
    N, inC, inH, inW, outC, kH, kW, dgr = 2, 4, 4, 4, 4, 3, 3, 1
    d = dict(dtype=torch.float64, device=DEV)
    inp = (torch.rand(N, inC, inH, inW, **d) * 0.01).requires_grad_()
    off = (torch.randn(N, dgr * 2 * kW * kH, inH, inW, **d) * 2).requires_grad_()
    mask = torch.sigmoid(torch.rand(N, dgr * kW * kH, inH, inW, **d)).detach().requires_grad_()
    wt = torch.randn(outC, inC // 2, kH, kW, **d).requires_grad_()
    bias = torch.rand(outC, **d).requires_grad_()
    assert torch.autograd.gradcheck(dcn.ModulatedDeformConvFunction.apply,
                                    (inp, off, mask, wt, bias, 1, 1, 1, 2, dgr, 1),
                                    eps=1e-6, atol=1e-5, rtol=1e-4, raise_exception=True,
                                    nondet_tol=1e-12)  # grad_input: an atomic scatter, as the reference's col2im


def test_dcn_rejects_float16_backward():
    x = torch.zeros((1, 1, 4, 4), dtype=torch.float16, device=DEV)
    w = torch.ones((1, 1, 3, 3), dtype=torch.float16, device=DEV)
    with pytest.raises(NotImplementedError):
        dcn.modulated_deform_conv_backward(x, w, None, torch.zeros((1, 18, 4, 4), dtype=torch.float16, device=DEV),
                                           torch.ones((1, 9, 4, 4), dtype=torch.float16, device=DEV), x,
                                           3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 64)
