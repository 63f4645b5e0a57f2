"""The section backward against gradients made by the REFERENCE's own autograd
(tests/golden/gen_golden.py bwd_* and gru_off_* cases: NLSPNModel.forward with grad on,
nlspnmodel.py:317-381, the offset branch through ModulatedDeformConvFunction
(modulated_deform_conv_func.py:15-56) with DCN's forward and backward stood in by a
float64 grid_sample definition and its autograd).

What these pin that the finite-difference checks of the oracle backward cannot tie to the
reference: the in-place TGASS/ASS clamp `aff_abs_sum[aff_abs_sum < 1.0] = 1.0` (:194, cuts
the gradient), `mask_fix.detach()` (:330), the clamp gradients (:361, :377), gamma's
gradient (:185), and GRU mode with learned offsets (the reference's forced default,
config.py:225-228) end to end, GRU-side weights included.

Loss: sum w_pred * pred + sum_t w_inter[t] * pred_inter[t] with the fixture's weights.
Bars (relative L2 per gradient tensor): 1e-4 for the section (the reference computes in
float32, the oracle in float64, the HIP path in float32 with float-atomic scatters);
GRU mode 1e-3 (its ConvGRU runs on MIOpen here and on CPU torch in the reference, so
last-bit differences enter the affinity every iteration; measured values in the asserts'
messages)."""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden

BWD = [n for n in golden_names("bwd_")]
FLAGS = {  # tests/golden/gen_golden.py BWD_CASES: (offset, affinity, preserve, clip, conf_prop)
    "bwd_off_tgass": (True, "TGASS", True, False, True),
    "bwd_off_tgass_clip": (True, "TGASS", True, True, True),
    "bwd_off_as": (True, "AS", True, False, True),
    "bwd_off_tc_noconf_nopreserve": (True, "TC", False, False, False),
    "bwd_nooff_tgass": (False, "TGASS", True, False, True),
    "bwd_nooff_ass_clip": (False, "ASS", True, True, True),
}
K = 8


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_fixture_set_complete():
    assert sorted(FLAGS) == BWD


def _f(z, k):
    return z[k].astype(np.float32)


@pytest.mark.parametrize("name", BWD)
def test_oracle_backward_matches_reference_autograd(oracle, name):
    """The fp64 oracle backward (oracle/nlspn_oracle_impl.h) against the reference's autograd."""
    z = load_golden(name)
    offset, kind, preserve, clip, conf = FLAGS[name]
    f64 = lambda k: _f(z, k).astype(np.float64)  # noqa: E731
    oa = f64("off_aff")
    ref = oracle.propagate_backward(
        f64("pred_init"), f64("dep"), f64("conf") if conf else None, oa[:, 2 * K:] if offset else oa,
        oa[:, :2 * K] if offset else None, float(z["gamma"][0]), f64("w_pred"), f64("w_inter"), kind=kind, kh=3, kw=3,
        prop_time=z["w_inter"].shape[0], preserve_input=preserve, always_clip=clip)
    g = z["g_off_aff"]
    checks = [("pred_init", ref["pred_init"], z["g_pred_init"]), ("aff", ref["aff"], g[:, 2 * K:] if offset else g)]
    if offset:
        checks.append(("offset", ref["offset"], g[:, :2 * K]))
    if conf:
        checks.append(("confidence", ref["confidence"], z["g_conf"]))
    for k, got, exp in checks:
        assert rel(got, exp) < 1e-4, (k, rel(got, exp))
    if "g_gamma" in z:
        assert abs(ref["gamma"] - float(z["g_gamma"][0])) <= 1e-4 * max(1.0, abs(float(z["g_gamma"][0])))


@pytest.mark.gpu
@pytest.mark.parametrize("name", BWD)
def test_gpu_backward_matches_reference_autograd(name):
    """propagate(...).backward() on the HIP path against the reference's autograd."""
    from nlspn_eccv20_amd import propagate
    dev = "cuda:0"
    z = load_golden(name)
    offset, kind, preserve, clip, conf = FLAGS[name]
    t = lambda k, rg=True: torch.from_numpy(np.ascontiguousarray(_f(z, k))).to(dev).requires_grad_(rg)  # noqa: E731
    oa, pi = t("off_aff"), t("pred_init")
    cf = t("conf") if conf else None
    T = z["w_inter"].shape[0]
    g = torch.tensor([float(z["gamma"][0])], device=dev, requires_grad=kind == "TGASS")
    o = propagate(pi, t("dep", False), cf, oa[:, 2 * K:] if offset else oa, oa[:, :2 * K] if offset else None, g,
                  prop_time=T, affinity=kind, kernel=(3, 3), preserve_input=preserve, always_clip=clip)
    loss = (o["pred"] * t("w_pred", False)).sum() + (o["pred_inter_tensor"] * t("w_inter", False)).sum()
    loss.backward()
    torch.cuda.synchronize()
    assert np.abs(o["pred"].detach().cpu().numpy() - z["pred"]).max() <= 1e-4
    ga = oa.grad.cpu().numpy()
    checks = [("pred_init", pi.grad.cpu().numpy(), z["g_pred_init"]), ("off_aff", ga, z["g_off_aff"])]
    if conf:
        checks.append(("confidence", cf.grad.cpu().numpy(), z["g_conf"]))
    for k, got, exp in checks:
        assert rel(got, exp) < 1e-4, (k, rel(got, exp))
    if "g_gamma" in z:
        gg = float(z["g_gamma"][0])
        assert abs(g.grad.item() - gg) <= 1e-4 * max(1.0, abs(gg)), (g.grad.item(), gg)


# ---------------------------------------------------------------- GRU mode + learned offsets
GRU_OFF = {"gru_off_tgass_preserve": dict(affinity="TGASS", preserve_input=True, always_clip=False, conf_prop=True)}


def _gru_off_model(name, dev):
    from nlspn_eccv20_amd import NLSPNModel
    from test_model_cpu import make_args
    z = load_golden(name)
    B, _, H, W = z["dep"].shape
    args = make_args(offset=True, use_GRU=True, use_S2D=False, prop_time=z["pred_inter"].shape[0], GRU_hidden_dim=8,
                     GRU_input_dim=8, zero_init_aff=False, patch_height=H, patch_width=W, **GRU_OFF[name])
    torch.manual_seed(0)
    m = NLSPNModel(args)
    sd = {k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd:")}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    return m.to(dev), z


def test_gru_offset_fixture_nontrivial():
    for name in GRU_OFF:
        z = load_golden(name)
        assert z["off_aff"].shape[1] == 3 * K and np.abs(z["off_aff"][:, :2 * K]).max() > 1.0
        assert any(k.startswith("gsd:GRU.") for k in z) and np.isfinite(z["g_off_aff"]).all()
        assert np.abs(z["offset"][:, 2 * (K // 2): 2 * (K // 2) + 2]).max() == 0.0  # _off_insert's zero reference tap


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GRU_OFF))
@pytest.mark.parametrize("grad", [False, True])
def test_gru_offset_matches_reference(name, grad):
    """NLSPNModel in GRU mode with learned offsets (propagate_heads) on the reference's
    weights and head outputs: outputs (inference and training paths) and, with grad, the
    gradients of pred_init, off_aff, confidence and every GRU-side weight."""
    dev = "cuda:0"
    m, z = _gru_off_model(name, dev)
    m.train(grad)
    t = lambda k, rg=False: torch.from_numpy(np.ascontiguousarray(z[k].astype(np.float32))).to(dev).requires_grad_(rg)  # noqa: E731
    with torch.set_grad_enabled(grad):
        pi, oa, cf = t("pred_init", grad), t("off_aff", grad), t("conf", grad)
        o = m.propagate_heads(pi, oa, cf, t("dep"))
        inter = torch.stack(list(o["pred_inter"]), 0)
    torch.cuda.synchronize()
    for got, key in ((inter, "pred_inter"), (o["pred"], "pred"), (o["aff"], "aff"), (o["offset"], "offset")):
        g = got.detach().cpu().numpy()
        err = float(np.sqrt(np.mean((g.astype(np.float64) - z[key]) ** 2)))
        assert err <= 1e-4 and np.abs(g - z[key]).max() <= 1e-3, (key, err)
    if not grad:
        return
    loss = (o["pred"] * t("w_pred")).sum() + (inter * t("w_inter")).sum()
    loss.backward()
    torch.cuda.synchronize()
    for key, got in (("g_pred_init", pi.grad), ("g_off_aff", oa.grad), ("g_conf", cf.grad)):
        e = rel(got.cpu().numpy(), z[key])
        assert e < 1e-3, (key, e)
    params = dict(m.named_parameters())
    n = 0
    for k, v in z.items():
        if k.startswith("gsd:"):
            p = params[k[4:]]
            assert p.grad is not None, k
            e = rel(p.grad.cpu().numpy(), v)
            assert e < 1e-3, (k, e)
            n += 1
    assert n >= 10
