"""Pin the CPU oracle (oracle/nlspn_oracle.c) before trusting it.

1. Against every golden vector the reference's own Python produced
   (tests/golden/gen_golden.py): affinity normalisation (4 kinds, K=8/24),
   _off_insert, the no-offset step, and the full T=18 propagation section.
2. The DCN (offset) branch has no runnable reference here (no CPU DCN in the
   reference; the CUDA extension cannot be built), so it is pinned through the
   reference's identities: zero offsets == no-offset branch in the
   interior, integer offsets == shifted reads, zero-offset DCN == plain stencil,
   and cross-checked against torch.nn.functional.grid_sample (an independent
   zero-padded bilinear sampler).
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden, loop_case_flags
from nlspn_eccv20_amd.synthetic import rmse, synth


@pytest.mark.parametrize("name", golden_names("affnorm_"))
def test_affinity_normalization_vs_reference(oracle, name):
    z = load_golden(name)
    kind = name.split("_")[1]
    out = oracle.affinity_normalization(z["aff_raw"], kind, float(z["gamma"][0]))
    # reference sums in ATen order, tanh from Sleef: a few ulp
    np.testing.assert_allclose(out, z["aff"], rtol=0, atol=5e-7)
    K = z["aff_raw"].shape[1]
    assert np.allclose(out[0, :, 5, 9], np.eye(K + 1)[K // 2])  # zero raw affinity -> identity taps


def test_off_insert_vs_reference(oracle):
    z = load_golden("off_insert_k8")
    np.testing.assert_array_equal(oracle.off_insert(z["off_raw"]), z["offset"])


def test_noffset_step_vs_reference(oracle):
    z = load_golden("step_noffset")
    np.testing.assert_allclose(oracle.prop_noffset(z["feat"], z["aff"]), z["out"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", golden_names("loop_"))
def test_propagation_loop_vs_reference(oracle, name):
    z = load_golden(name)
    kind, preserve, clip = loop_case_flags(name)
    o = oracle.propagate(z["pred_init"], z["dep"], z.get("conf"), z["aff_raw"], None, float(z["gamma"][0]),
                         kind=kind, preserve_input=preserve, always_clip=clip)
    assert rmse(o["pred"], z["pred"]) < 1e-6
    np.testing.assert_allclose(o["pred"], z["pred"], rtol=0, atol=1e-5)
    if "pred_inter" in z:
        np.testing.assert_allclose(o["pred_inter"], z["pred_inter"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(o["aff"], z["aff"], rtol=0, atol=1e-6)
    else:
        np.testing.assert_allclose(o["pred_inter"][-1], z["pred_inter_last"], rtol=0, atol=1e-5)
    if "confidence" in z:
        np.testing.assert_array_equal(o["confidence"], z["confidence"])


def test_f32_tracks_f64(oracle):
    s = synth(2, 32, 40, 8, seed=1)
    aff, off = s["off_aff"][:, 16:], s["off_aff"][:, :16]
    o32 = oracle.propagate(s["pred_init"], s["dep"], s["conf"], aff, off, 4.0)
    o64 = oracle.propagate(*(x.astype(np.float64) for x in (s["pred_init"], s["dep"], s["conf"], aff, off)), 4.0)
    assert rmse(o32["pred"], o64["pred"]) < 1e-5


def _zero_offset_vs_noffset(oracle, H, W, seed):
    rng = np.random.default_rng(seed)
    feat = rng.uniform(0, 10, (2, 1, H, W)).astype(np.float32)
    aff = oracle.affinity_normalization(np.abs(rng.standard_normal((2, 8, H, W))).astype(np.float32), "TGASS", 4.0)
    off = np.zeros((2, 18, H, W), np.float32)
    a = oracle.mdcn_c1(feat, off, aff)
    b = oracle.prop_noffset(feat, aff)
    return a, b


def test_zero_offset_dcn_equals_noffset_interior(oracle):
    a, b = _zero_offset_vs_noffset(oracle, 12, 17, 3)
    np.testing.assert_array_equal(a[..., 1:-1, 1:-1], b[..., 1:-1, 1:-1])  # SURVEY §4 identity 2
    assert np.abs(a - b).max() > 0  # borders differ: zero vs replicate padding


def test_integer_offsets_are_shifted_reads(oracle):
    rng = np.random.default_rng(5)
    H, W = 10, 13
    im = rng.uniform(0, 1, (1, 1, H, W)).astype(np.float32)
    off = np.zeros((1, 18, H, W), np.float32)
    mask = np.zeros((1, 9, H, W), np.float32)
    off[0, 0], off[0, 1] = 2.0, -3.0  # tap 0 base (-1,-1) -> shift (+1, -4)
    mask[0, 0] = 1.0
    out = oracle.mdcn_c1(im, off, mask)
    exp = np.zeros((H, W), np.float32)
    for y in range(H):
        for x in range(W):
            yy, xx = y + 1, x - 4
            if 0 <= yy < H and 0 <= xx < W:
                exp[y, x] = im[0, 0, yy, xx]
    np.testing.assert_array_equal(out[0, 0], exp)


@pytest.mark.parametrize("kh,kw,sigma", [(3, 3, 2.0), (3, 3, 50.0), (5, 5, 2.0), (1, 17, 3.0)])
def test_dcn_matches_grid_sample(oracle, kh, kw, sigma):
    """Independent bilinear sampler: grid_sample(zeros padding, align_corners=True)."""
    rng = np.random.default_rng(11)
    B, H, W, KK = 2, 11, 19, kh * kw
    im = rng.uniform(0, 10, (B, 1, H, W)).astype(np.float64)
    off = (rng.standard_normal((B, 2 * KK, H, W)) * sigma).astype(np.float64)
    mask = rng.standard_normal((B, KK, H, W)).astype(np.float64)
    out = oracle.mdcn_c1(im, off, mask, kh, kw)
    ph, pw = (kh - 1) // 2, (kw - 1) // 2
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    ref = np.zeros((B, 1, H, W))
    for t in range(KK):
        i, j = divmod(t, kw)
        hs = yy - ph + i + off[:, 2 * t]
        ws = xx - pw + j + off[:, 2 * t + 1]
        grid = np.stack([2 * ws / (W - 1) - 1, 2 * hs / (H - 1) - 1], -1)
        v = torch.nn.functional.grid_sample(torch.from_numpy(im), torch.from_numpy(grid), mode="bilinear",
                                            padding_mode="zeros", align_corners=True).numpy()
        ref += v * mask[:, t:t + 1]
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9)


def test_zero_offset_dcn_is_plain_stencil(oracle):
    """deformconv/test.py:69-110 analogue: zero offsets, mask 1 -> the fixed 3x3 stencil
    (conv2d with all-ones weights, zero padding)."""
    rng = np.random.default_rng(2)
    im = rng.standard_normal((2, 1, 6, 7)).astype(np.float64)
    out = oracle.mdcn_c1(im, np.zeros((2, 18, 6, 7)), np.ones((2, 9, 6, 7)))
    ref = torch.nn.functional.conv2d(torch.from_numpy(im), torch.ones(1, 1, 3, 3, dtype=torch.float64), padding=1)
    np.testing.assert_allclose(out, ref.numpy(), rtol=0, atol=1e-12)


def test_oracle_rejects_bad_geometry(oracle):
    z = synth(1, 4, 4, 8, offset=False)
    with pytest.raises(ValueError):
        oracle.propagate(z["pred_init"], z["dep"], z["conf"], np.zeros((1, 24, 4, 4), np.float32), None, 1.0,
                         kh=5, kw=5)  # no-offset branch is 3x3 only (nlspnmodel.py:213-221)
