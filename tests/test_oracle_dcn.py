"""CPU: the oracle's generic modulated DCNv2 (seam 2, `DCN` module, vision.cpp:9-10),
pinned before it is used to check the HIP kernels.

Pins (no runnable reference DCN exists here: CPU DCN absent, CUDA extension
unbuildable — DESIGN.md §4):
  * C = Cout = 1, weight 1, bias 0 reduces to the NLSPN specialisation mdcn_c1
    (bit-exact: same operation order);
  * zero offsets and unit mask reduce to a grouped conv2d (the reference's own
    check, deformconv/test.py:69-110), against torch in float64;
  * the backward against central finite differences of the float64 forward, for
    every gradient (grad_input with square padding, where the reference's
    col2im pad_w := pad_h quirk, .cuh:371, does not apply).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F


def _rand_case(rng, B, C, H, W, Cout, kh, kw, group, dg, stride=(1, 1), pad=(1, 1), dil=(1, 1), sigma=1.5,
               dtype=np.float64):
    Ho = (H + 2 * pad[0] - (dil[0] * (kh - 1) + 1)) // stride[0] + 1
    Wo = (W + 2 * pad[1] - (dil[1] * (kw - 1) + 1)) // stride[1] + 1
    inp = rng.standard_normal((B, C, H, W)).astype(dtype)
    wt = rng.standard_normal((Cout, C // group, kh, kw)).astype(dtype)
    bias = rng.standard_normal((Cout,)).astype(dtype)
    off = (rng.standard_normal((B, 2 * dg * kh * kw, Ho, Wo)) * sigma).astype(dtype)
    # keep sample points away from integer grid lines (finite differences across a
    # bilinear kink are not derivatives)
    frac = off - np.floor(off)
    off = np.where(np.abs(frac - 0.5) > 0.45, off + 0.2, off)
    mask = rng.random((B, dg * kh * kw, Ho, Wo)).astype(dtype)
    return inp, wt, bias, off, mask


def test_generic_equals_nlspn_specialisation(oracle):
    rng = np.random.default_rng(1)
    inp, _, _, off, mask = _rand_case(rng, 2, 1, 9, 11, 1, 3, 3, 1, 1, dtype=np.float32)
    w = np.ones((1, 1, 3, 3), np.float32)
    a = oracle.mdcn_forward(inp, w, np.zeros(1, np.float32), off, mask)
    b = oracle.mdcn_c1(inp, off, mask)
    np.testing.assert_array_equal(a, b + np.float32(0))


@pytest.mark.parametrize("C,Cout,group,stride,pad,dil", [
    (4, 6, 2, (1, 1), (1, 1), (1, 1)),
    (3, 3, 1, (2, 1), (1, 2), (1, 1)),
    (4, 4, 4, (1, 1), (2, 2), (2, 2)),
])
def test_zero_offset_is_grouped_conv(oracle, C, Cout, group, stride, pad, dil):
    rng = np.random.default_rng(C * 7 + Cout)
    inp, wt, bias, off, mask = _rand_case(rng, 2, C, 8, 10, Cout, 3, 3, group, 1, stride, pad, dil)
    off[:] = 0
    mask[:] = 1
    out = oracle.mdcn_forward(inp, wt, bias, off, mask, stride, pad, dil, group, 1)
    ref = F.conv2d(torch.from_numpy(inp), torch.from_numpy(wt), torch.from_numpy(bias), stride, pad, dil, group)
    np.testing.assert_allclose(out, ref.numpy(), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("C,Cout,group,dg,kh,kw,stride,pad,dil", [
    (1, 1, 1, 1, 3, 3, (1, 1), (1, 1), (1, 1)),   # NLSPN shape
    (4, 2, 2, 2, 3, 3, (1, 1), (1, 1), (1, 1)),   # groups and deformable groups
    (2, 3, 1, 1, 3, 3, (2, 2), (1, 1), (1, 1)),   # stride
    (2, 2, 1, 2, 3, 3, (1, 1), (2, 2), (2, 2)),   # dilation
    (1, 1, 1, 1, 5, 5, (1, 1), (2, 2), (1, 1)),   # 5x5
])
def test_backward_finite_differences(oracle, C, Cout, group, dg, kh, kw, stride, pad, dil):
    rng = np.random.default_rng(C * 100 + Cout * 10 + dg)
    B, H, W = 1, 6, 7
    inp, wt, bias, off, mask = _rand_case(rng, B, C, H, W, Cout, kh, kw, group, dg, stride, pad, dil)
    fwd = lambda i, w, b, o, m: oracle.mdcn_forward(i, w, b, o, m, stride, pad, dil, group, dg)  # noqa: E731
    out = fwd(inp, wt, bias, off, mask)
    go = rng.standard_normal(out.shape)
    gi, goff, gm, gw, gb = oracle.mdcn_backward(inp, wt, off, mask, go, stride, pad, dil, group, dg)
    loss = lambda *a: float(np.sum(fwd(*a) * go))  # noqa: E731
    args = [inp, wt, bias, off, mask]
    grads = [gi, gw, gb, goff, gm]
    eps = 1e-6
    for which, g in enumerate(grads):
        x = args[which]
        idx = rng.choice(x.size, size=min(12, x.size), replace=False)
        for k in idx:
            xp = x.copy().reshape(-1)
            xm = x.copy().reshape(-1)
            xp[k] += eps
            xm[k] -= eps
            ap, am = list(args), list(args)
            ap[which] = xp.reshape(x.shape)
            am[which] = xm.reshape(x.shape)
            fd = (loss(*ap) - loss(*am)) / (2 * eps)
            np.testing.assert_allclose(g.reshape(-1)[k], fd, rtol=1e-5, atol=1e-7,
                                       err_msg=f"grad {['input', 'weight', 'bias', 'offset', 'mask'][which]}[{k}]")
