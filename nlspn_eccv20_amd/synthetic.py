"""Seeded synthetic propagation inputs, numpy; used by tests and bench.py.

pred_init ~ U(0, max_depth); dep = U(0, max_depth) * Bernoulli(density);
conf ~ U(0, 1); raw affinity = |N(0, 1)| (convex operator) or N(0, 1) (signed);
offsets ~ N(0, off_sigma^2) px.  Affinity and offsets are packed like the
reference head output off_aff (B, 3K, H, W) = [offsets 2K | affinity K]
(nlspnmodel.py:301-305).
"""
import numpy as np


def synth(B, H, W, K, seed=7240, density=0.05, max_depth=10.0, off_sigma=2.0, signed=False, offset=True):
    rng = np.random.default_rng(seed)
    f32 = np.float32
    pred_init = rng.uniform(0, max_depth, (B, 1, H, W)).astype(f32)
    dep = (rng.uniform(0, max_depth, (B, 1, H, W)) * (rng.random((B, 1, H, W)) < density)).astype(f32)
    conf = rng.random((B, 1, H, W)).astype(f32)
    aff = rng.standard_normal((B, K, H, W)).astype(f32)
    if not signed:
        aff = np.abs(aff)
    if offset:
        off = (rng.standard_normal((B, 2 * K, H, W)) * off_sigma).astype(f32)
        off_aff = np.concatenate([off, aff], 1)
    else:
        off_aff = aff
    return {"pred_init": pred_init, "dep": dep, "conf": conf, "off_aff": np.ascontiguousarray(off_aff), "K": K}


def split(off_aff, K, offset=True):
    if offset:
        return off_aff[:, 2 * K:], off_aff[:, :2 * K]
    return off_aff, None


def rmse(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)))
