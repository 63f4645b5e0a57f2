"""The offset (DCN) branch against the reference's own forward (verdict r2 item 3).

tests/golden/offloop_*.npz come from the reference's NLSPNModel.forward with
offset=True (src/model/nlspnmodel.py:317-383), whose _propagate_once calls
ModulatedDeformConvFunction.apply (:204-208 -> modulated_deform_conv_func.py:26-34 ->
DCN.modulated_deform_conv_forward).  The CUDA extension cannot be built here, so
gen_golden.py gives the `DCN` stub a forward written from the DCNv2 definition on
torch.grid_sample (float64, independent of oracle/).  The fixtures therefore pin the
reference-side plumbing of the branch — _off_insert's channel layout feeding the DCN's
2t / 2t+1 channels, the normalised affinity as the mask, self.padding, weight / bias,
the loop order and the blends — for 3x3 and 5x5, offsets N(0, 2^2) and N(0, 50^2),
always_clip on and off.

CPU: the oracle restatement against them.  GPU: the HIP section (nlspn_propagate)
against them, at the north-star bar (RMSE <= 1e-4 on fp32 depth).  The stand-in rounds
once in float64 where the reference's CUDA kernel and ours round per float32 operation,
and TGASS/TC take tanh from different libraries: a few 1e-7 of difference is expected.
"""
import numpy as np
import pytest

from conftest import load_golden
from nlspn_eccv20_amd.synthetic import rmse

# name -> (prop_kernel, affinity, preserve_input, always_clip, conf_prop); gen_golden.OFFSET_CASES
OFFLOOP = {
    "offloop_k3_s2_tgass": (3, "TGASS", True, False, True),
    "offloop_k3_s2_ass_clip_noconf": (3, "ASS", True, True, False),
    "offloop_k3_s50_tgass_clip": (3, "TGASS", True, True, True),
    "offloop_k5_s2_tgass": (5, "TGASS", True, False, True),
    "offloop_k5_s50_tc_nopreserve": (5, "TC", False, False, True),
}
KEEP = (0, 8, 17)  # gen_golden.OFFLOOP_KEEP
ORACLE_RMSE, ORACLE_MAX = 2e-6, 2e-5
GPU_RMSE, GPU_MAX = 1e-4, 1e-3  # the north-star bar; measured values are far below (printed)


def _inputs(z, k):
    f = lambda a: np.ascontiguousarray(a.astype(np.float32))  # noqa: E731  (float16-exact values)
    K = k * k - 1
    oa = f(z["off_aff"])
    return (f(z["pred_init"]), f(z["dep"]), f(z["conf"]) if "conf" in z else None, oa[:, 2 * K:], oa[:, :2 * K],
            float(z["gamma"][0]))


def _check(name, pred, inter_sel, offset, z, tol_rmse, tol_max):
    errs = [rmse(pred, z["pred"])] + [rmse(inter_sel[i], z["pred_inter_sel"][i]) for i in range(len(KEEP))]
    mx = max(float(np.abs(pred - z["pred"]).max()), float(np.abs(inter_sel - z["pred_inter_sel"]).max()))
    print(f"{name}: rmse pred {errs[0]:.2e}, inter {max(errs[1:]):.2e}, max {mx:.2e}")
    assert max(errs) <= tol_rmse and mx <= tol_max, (errs, mx)
    np.testing.assert_array_equal(offset, z["offset"].astype(np.float32))  # _off_insert layout, exact


@pytest.mark.parametrize("name", sorted(OFFLOOP))
def test_oracle_offset_loop_vs_reference(oracle, name):
    k, kind, pre, clip, _ = OFFLOOP[name]
    z = load_golden(name)
    pi, dep, conf, aff, off, g = _inputs(z, k)
    o = oracle.propagate(pi, dep, conf, aff, off, g, kind=kind, kh=k, kw=k, prop_time=18, preserve_input=pre,
                         always_clip=clip)
    _check(name, o["pred"], o["pred_inter"][list(KEEP)], o["offset"], z, ORACLE_RMSE, ORACLE_MAX)
    if "confidence" in z:
        np.testing.assert_array_equal(o["confidence"], z["confidence"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(OFFLOOP))
def test_hip_offset_loop_vs_reference(name):
    import torch

    from nlspn_eccv20_amd import propagate
    k, kind, pre, clip, _ = OFFLOOP[name]
    z = load_golden(name)
    pi, dep, conf, aff, off, g = _inputs(z, k)
    t = lambda a: None if a is None else torch.from_numpy(a).to("cuda:0")  # noqa: E731
    with torch.no_grad():
        o = propagate(t(pi), t(dep) if pre else None, t(conf), t(aff), t(off), torch.tensor([g], device="cuda:0"),
                      prop_time=18, affinity=kind, kernel=(k, k), preserve_input=pre, always_clip=clip)
    torch.cuda.synchronize()
    inter = o["pred_inter_tensor"].cpu().numpy()[list(KEEP)]
    _check(name, o["pred"].cpu().numpy(), inter, o["offset"].cpu().numpy(), z, GPU_RMSE, GPU_MAX)
    if "confidence" in z:
        assert np.array_equal(o["confidence"].cpu().numpy(), z["confidence"])
