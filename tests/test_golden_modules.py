"""GRU mode and the S2D front against fixtures made by the REFERENCE's own modules
(tests/golden/gen_golden.py, gru_* / s2d_* cases: NLSPNModel.forward with
use_GRU=True, nlspnmodel.py:365-373 + ConvGRU :386-403 + _aff_head/_clip_as
:228-250; S2D.forward :406-462), not against a restatement of them.

Each fixture holds the inputs, the reference's outputs and the reference module's
weights (keys "sd:<state_dict name>"), so the drop-in loads the very same weights.

Bars:
  * S2D pool pyramid: bit-exact (min/max are exact in any order), CPU oracle and the
    HIP kernel alike; the 32-channel output (two 1x1 layers + the 3x3 conv, summation
    order differs between CPU torch, the oracle and MIOpen): max |diff| <= 1e-4.
  * GRU mode, every iteration's depth and the final affinity: RMSE <= 1e-4 (the
    north-star bar) and max |diff| <= 1e-3 — the GRU convolutions run on MIOpen here
    and on CPU torch in the reference, so last-bit differences enter the affinity
    each iteration.
"""
import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import NLSPNModel
from nlspn_eccv20_amd.model import S2D

from conftest import load_golden
from test_model_cpu import make_args

GRU_FLAGS = {  # tests/golden/gen_golden.py GRU_CASES
    "gru_tgass_preserve": dict(affinity="TGASS", preserve_input=True, always_clip=False, conf_prop=True),
    "gru_ass_clip_noconf": dict(affinity="ASS", preserve_input=True, always_clip=True, conf_prop=False),
}
S2D_CASES = ("s2d_20x28", "s2d_13x17")


def _sd(z):
    return {k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd:")}


def _s2d_module(z, dev="cpu"):
    m = S2D()
    m.load_state_dict(_sd(z), strict=True)
    return m.to(dev).eval()


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("name", S2D_CASES)
def test_s2d_cpu_module_matches_reference(name):
    """The drop-in S2D module's CPU path (the reference's torch ops, restated) on the
    reference's weights and inputs."""
    z = load_golden(name)
    m = _s2d_module(z)
    with torch.no_grad():
        out = m(torch.from_numpy(z["dep"]))
    assert np.abs(out.numpy() - z["out"]).max() <= 1e-4


@pytest.mark.parametrize("name", S2D_CASES)
def test_s2d_oracle_pyramid_matches_reference(name):
    """The oracle's pool pyramid (oracle.s2d_front) bit-exact against the pyramid the
    reference's pools produced (captured at pool_convs' input)."""
    from oracle import oracle as O
    z = load_golden(name)
    sd = _sd(z)
    args = [z["dep"]] + [sd[k].numpy() for k in ("pool_convs.0.0.weight", "pool_convs.0.0.bias",
                                                 "pool_convs.1.0.weight", "pool_convs.1.0.bias")]
    out17, pyr = O.s2d_front(*args)
    assert np.array_equal(pyr, z["pyramid"])
    assert np.array_equal(out17[:, 16], z["dep"][:, 0])


def test_gru_fixtures_are_nontrivial():
    """The GRU really re-estimated the affinity (not the head's affinity all along)."""
    for name, kw in GRU_FLAGS.items():
        z = load_golden(name)
        sd = _sd(z)
        assert any(k.startswith("GRU.") for k in sd) and any(k.startswith("decode_aff.") for k in sd)
        assert z["pred_inter"].shape[0] == 6 and np.isfinite(z["pred"]).all()
        # the final affinity is the GRU head's, so it differs from the normalised raw one
        raw = torch.from_numpy(z["aff_raw"])
        assert z["aff"].shape == (raw.shape[0], 9) + raw.shape[2:]
        assert np.abs(z["aff"][:, :4] - raw.numpy()[:, :4]).max() > 1e-3


# ------------------------------------------------------------------ GPU
def _gru_model(name, dev):
    z = load_golden(name)
    kw = GRU_FLAGS[name]
    B, _, H, W = z["dep"].shape
    args = make_args(offset=False, use_GRU=True, use_S2D=False, prop_time=z["pred_inter"].shape[0],
                     GRU_hidden_dim=8, GRU_input_dim=8, zero_init_aff=False, patch_height=H, patch_width=W, **kw)
    torch.manual_seed(0)
    m = NLSPNModel(args)
    missing, unexpected = m.load_state_dict(_sd(z), strict=False)
    assert not unexpected, unexpected
    loaded = set(_sd(z))
    assert loaded and all(k in dict(m.named_parameters()) or k in dict(m.named_buffers()) for k in loaded)
    return m.to(dev).eval(), z


def _rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GRU_FLAGS))
@pytest.mark.parametrize("grad", [False, True])
def test_gru_mode_matches_reference(name, grad):
    """NLSPNModel GRU mode (prop_step per iteration between MIOpen ConvGRU steps) on the
    reference's weights and head outputs, inference path and training path."""
    dev = "cuda:0"
    m, z = _gru_model(name, dev)
    t = lambda k: torch.from_numpy(z[k]).to(dev)  # noqa: E731
    conf = t("conf") if "conf" in z else None
    with torch.set_grad_enabled(grad):
        pi = t("pred_init").requires_grad_(grad)
        o = m.propagate_heads(pi, t("aff_raw"), conf, t("dep"))
    torch.cuda.synchronize()
    got_inter = np.stack([p.detach().cpu().numpy() for p in o["pred_inter"]])
    assert got_inter.shape == z["pred_inter"].shape
    for got, ref in ((got_inter, z["pred_inter"]), (o["pred"].detach().cpu().numpy(), z["pred"]),
                     (o["aff"].detach().cpu().numpy(), z["aff"])):
        assert _rmse(got, ref) <= 1e-4 and np.abs(got - ref).max() <= 1e-3
    if "confidence" in z:
        assert np.abs(o["confidence"].detach().cpu().numpy() - z["confidence"]).max() <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("name", S2D_CASES)
def test_s2d_kernel_matches_reference(name):
    """The fused S2D front (HIP) + MIOpen 3x3 conv on the reference's weights: pyramid
    bit-exact, output to 1e-4."""
    from nlspn_eccv20_amd.s2d import _run
    dev = "cuda:0"
    z = load_golden(name)
    m = _s2d_module(z, dev)
    dep = torch.from_numpy(z["dep"]).to(dev)
    c0, c1 = m.pool_convs[0][0], m.pool_convs[1][0]
    with torch.no_grad():
        out17, pyr = _run(dep, c0.weight, c0.bias, c1.weight, c1.bias, want_pyr=True)
        out = m(dep)
    torch.cuda.synchronize()
    assert np.array_equal(pyr.cpu().numpy(), z["pyramid"])
    assert np.abs(out.cpu().numpy() - z["out"]).max() <= 1e-4
