"""GPU parity of one fused step with fp16 storage (the C5 step kernel's MIX path: fp16 planes
read through v_fma_mix_f32, out-of-image window cells loaded as zeros from an out-of-range
buffer offset) and of the exact h == -1 / w == -1 taps of edge tiles.

fp16 storage, one step: BIT-EXACT vs the fp32 oracle on the same fp16 values, rounded to
fp16.  An fp16 x fp16 product and an fp16 -> fp32 conversion are exact, so the kernel's
fp32 arithmetic on fp16 inputs is the oracle's fp32 arithmetic on those values; the
reference tap's weight is 1 - (sum of the fp16 affinities in tap order) in fp32, so the
oracle is given that plane (nlspnmodel.py:262-263).
Reference: modulated_deform_im2col_cuda.cuh:127-194 (sampling, validity test :180).
"""
import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import prop_step
from nlspn_eccv20_amd.synthetic import synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def cu(x, dtype=torch.float32):
    return None if x is None else torch.from_numpy(np.ascontiguousarray(x)).to(DEV, dtype)


def host(t):
    return t.detach().float().cpu().numpy()


def f16(x):
    return x.astype(np.float16).astype(np.float32)


def _inputs(oracle, B, H, W, kh, kw, sigma, seed, half):
    K = kh * kw - 1
    s = synth(B, H, W, K, seed=seed, off_sigma=sigma)
    aff = oracle.affinity_normalization(s["off_aff"][:, 2 * K:], "TGASS", 0.5 * K)
    off_ins = oracle.off_insert(s["off_aff"][:, :2 * K])
    conf = s["conf"].copy()
    conf[s["dep"] > 0] = 1.0
    p, dep = s["pred_init"], s["dep"]
    if half:
        p, dep, conf, aff, off_ins = (f16(x) for x in (p, dep, conf, aff, off_ins))
    ref = K // 2
    acc = np.zeros((B, H, W), np.float32)
    for k in range(K + 1):
        if k != ref:
            acc = acc + aff[:, k]
    aff[:, ref] = np.float32(1.0) - acc  # the kernel's reference-tap weight, same order
    return p, dep, conf, aff, off_ins


def _oracle_step(oracle, p, conf, dep, aff, off_ins, kh, kw):
    f = p * conf if conf is not None else p
    out = oracle.mdcn_c1(f, off_ins, aff, kh, kw)
    m = (dep > 0).astype(np.float32)
    return (np.float32(1.0) - m) * out + m * dep


@pytest.mark.parametrize("B,H,W,kh,kw,sigma", [
    (2, 30, 72, 1, 17, 3.0),     # C5 geometry, window hits
    (1, 64, 128, 1, 17, 12.0),   # many taps beyond the LDS halo -> global fallback
    (2, 33, 64, 1, 17, 60.0),    # mostly out-of-image taps
    (2, 40, 56, 3, 3, 2.0),      # 3x3 fp16
    (1, 21, 40, 5, 5, 4.0),      # K=24 fp16
])
@pytest.mark.parametrize("with_conf", [True, False])
def test_step_fp16_bitexact_vs_oracle(oracle, B, H, W, kh, kw, sigma, with_conf):
    p, dep, conf, aff, off_ins = _inputs(oracle, B, H, W, kh, kw, sigma, seed=B * H + W + kw, half=True)
    if not with_conf:
        conf = None
    exp = _oracle_step(oracle, p, conf, dep, aff, off_ins, kh, kw).astype(np.float16)
    h = torch.float16
    out = prop_step(cu(p, h), cu(conf, h), cu(dep, h), cu(aff, h), cu(off_ins, h), kernel=(kh, kw))
    assert out.dtype == h
    np.testing.assert_array_equal(out.cpu().numpy(), exp)


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("kh,kw,axis", [(1, 17, "h"), (1, 17, "w"), (3, 3, "h"), (3, 3, "w")])
def test_exact_minus_one_tap_ignores_nonfinite_edge_cells(oracle, half, kh, kw, axis):
    """A tap at exactly h == -1 (or w == -1) is invalid (.cuh:180: h_im > -1 fails): val = 0,
    even when the in-image row (column) its footprint touches with weight 0 holds inf —
    the window's zero padding alone would give 0 * inf = NaN."""
    H, W = 24, 64
    p, dep, conf, aff, off_ins = _inputs(oracle, 1, H, W, kh, kw, 2.0, seed=31, half=half)
    dep[:] = 0.0  # no preserve blend over the probed pixels
    K = kh * kw - 1
    ph, pw = (kh - 1) // 2, (kw - 1) // 2
    t = 0  # first tap: i = 0, j = 0
    if axis == "h":  # pixel (0, x0): h = 0 - ph + 0 + dh = -1 exactly, w = x0 - pw + dw -> cells (0, x0+4), (0, x0+5)
        y0, x0 = 0, 20
        off_ins[0, 2 * t, y0, x0] = ph - 1.0
        off_ins[0, 2 * t + 1, y0, x0] = pw + 4.5
        bad = (0, x0 + 5)
    else:            # pixel (y0, 0): w = -1 exactly, h = y0 - ph + dh -> cells (y0+4, 0), (y0+5, 0)
        y0, x0 = 6, 0
        off_ins[0, 2 * t, y0, x0] = ph + 4.5
        off_ins[0, 2 * t + 1, y0, x0] = pw - 1.0
        bad = (y0 + 5, 0)
    p[0, 0][bad] = np.inf
    exp = _oracle_step(oracle, p, conf, dep, aff, off_ins, kh, kw)
    dt = torch.float16 if half else torch.float32
    out = host(prop_step(cu(p, dt), cu(conf, dt), cu(dep, dt), cu(aff, dt), cu(off_ins, dt), kernel=(kh, kw)))
    if half:
        exp = exp.astype(np.float16).astype(np.float32)
    assert np.isfinite(exp[0, 0, y0, x0]) and np.isfinite(out[0, 0, y0, x0])
    # everywhere, NaNs included: the inf cell's left / upper neighbours read it through
    # their zero-offset reference tap with weight 0 in the reference's four-corner form
    # (.cuh:37-52: 0 * inf = NaN), and so does the kernel once the window holds a
    # non-finite f
    np.testing.assert_array_equal(out[0, 0], exp[0, 0])
    by, bx = bad
    for ny, nx in ((by, bx - 1), (by - 1, bx), (by - 1, bx - 1)):
        if ny >= 0 and nx >= 0:
            assert np.isnan(out[0, 0, ny, nx]) and np.isnan(exp[0, 0, ny, nx]), (ny, nx)
    assert K > 0
