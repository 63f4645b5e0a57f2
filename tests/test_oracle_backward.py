"""Pin the oracle's backward (oracle/nlspn_oracle_impl.h orc_propagate_backward) against
central finite differences of the oracle forward in fp64 — the forward itself being
pinned to the reference (tests/test_oracle.py).  This plays the role of the
reference's own gradcheck (src/model/deformconv/test.py:405-434) for the whole
propagation section: DCN backward (col2im / col2im_coord) plus autograd of the
affinity normalisation, blends and clamps."""
import numpy as np
import pytest

from nlspn_eccv20_amd.synthetic import synth

EPS = 1e-6


def _loss_and_weights(seed, B, H, W, T):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((B, 1, H, W)), rng.standard_normal((T, B, 1, H, W))


def _fd_check(oracle, s, kw, T, names, n_probe=12, seed=0):
    K = s["K"]
    f64 = lambda x: None if x is None else x.astype(np.float64)  # noqa: E731
    inp = {"pred_init": f64(s["pred_init"]), "dep": f64(s["dep"]), "conf": f64(s["conf"]),
           "aff": f64(s["off_aff"][:, 2 * K:]) if kw.get("offset", True) else f64(s["off_aff"]),
           "off": f64(s["off_aff"][:, :2 * K]) if kw.get("offset", True) else None}
    gamma = kw.get("gamma", 0.5 * K)
    okw = dict(kind=kw.get("kind", "TGASS"), kh=kw.get("kh", 3), kw=kw.get("kw", 3), prop_time=T,
               preserve_input=kw.get("preserve", True), always_clip=kw.get("clip", False))
    B, _, H, W = inp["pred_init"].shape
    wp, wi = _loss_and_weights(seed, B, H, W, T)

    def loss(d, g):
        o = oracle.propagate(d["pred_init"], d["dep"], d["conf"], d["aff"], d["off"], g, **okw)
        return float((o["pred"] * wp).sum() + (o["pred_inter"] * wi).sum())

    gr = oracle.propagate_backward(inp["pred_init"], inp["dep"], inp["conf"], inp["aff"], inp["off"], gamma,
                                   wp, wi, **okw)
    key = {"pred_init": "pred_init", "conf": "confidence", "aff": "aff", "off": "offset"}
    rng = np.random.default_rng(seed + 1)
    for name in names:
        if name == "gamma":
            num = (loss(inp, gamma + EPS) - loss(inp, gamma - EPS)) / (2 * EPS)
            assert abs(num - gr["gamma"]) <= 1e-5 * max(1.0, abs(num)), (num, gr["gamma"])
            continue
        arr, g = inp[name], gr[key[name]]
        for _ in range(n_probe):
            idx = tuple(rng.integers(0, n) for n in arr.shape)
            old = arr[idx]
            arr[idx] = old + EPS
            lp = loss(inp, gamma)
            arr[idx] = old - EPS
            lm = loss(inp, gamma)
            arr[idx] = old
            num = (lp - lm) / (2 * EPS)
            assert abs(num - g[idx]) <= 1e-5 * max(1.0, abs(num)), (name, idx, num, g[idx])


@pytest.mark.parametrize("kw", [
    dict(),                                   # TGASS, preserve, learned offsets
    dict(clip=True),
    dict(preserve=False),
    dict(kind="ASS", gamma=1.0),
    dict(kind="AS", gamma=1.0),
    dict(kind="TC", gamma=8.0),
    dict(offset=False),                       # no-offset replicate branch
    dict(kh=1, kw=17, gamma=8.0),             # K=16 geometry
])
def test_backward_matches_finite_differences(oracle, kw):
    K = kw.get("kh", 3) * kw.get("kw", 3) - 1
    s = synth(1, 6, 7, K, seed=3, density=0.15, off_sigma=1.3, offset=kw.get("offset", True))
    names = ["pred_init", "conf", "aff"] + (["off"] if kw.get("offset", True) else [])
    if kw.get("kind", "TGASS") == "TGASS":
        names.append("gamma")
    _fd_check(oracle, s, kw, 3, names)
