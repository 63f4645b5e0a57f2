"""Replays of summary dumps (nlspn_eccv20_amd.replay) on the HIP path.

* no-offset dumps built from the reference's own loop fixtures (its normalised 'aff'
  and gamma, as nlspnsummary.py:265-268 would save them) replay to the reference's
  pred_inter / pred (the loop fixtures' tolerance: RMSE < 1e-5, max 1e-4);
* offset dumps written by save_dump from propagate()'s output replay bit-exactly to
  that output (fp32: same planes, same IEEE sequence);
* a 1x17 fp16 dump (config C5's geometry) replays within the fp16 bar (RMSE <= 1e-2)
  of its fp32 replay.
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden, loop_case_flags
from nlspn_eccv20_amd import propagate
from nlspn_eccv20_amd.replay import load_dump, replay, save_dump
from nlspn_eccv20_amd.synthetic import rmse, synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def host(t):
    return t.detach().float().cpu().numpy()


@pytest.mark.parametrize("name", [n for n in golden_names("loop_") if n != "loop_tgass_40x56"])
def test_replay_no_offset_dump_vs_reference(name, tmp_path):
    z = load_golden(name)
    kind, preserve, clip = loop_case_flags(name)
    save_dump(str(tmp_path), {"aff": torch.from_numpy(z["aff"]), "offset": None,
                              "gamma": torch.from_numpy(z["gamma"])})
    o = replay(load_dump(str(tmp_path)), z["pred_init"], z["dep"], z.get("conf"), prop_time=18,
               preserve_input=preserve, always_clip=clip, device=DEV)
    torch.cuda.synchronize()
    assert rmse(host(o["pred"]), z["pred"]) < 1e-5
    np.testing.assert_allclose(host(o["pred"]), z["pred"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(host(o["pred_inter_tensor"]), z["pred_inter"], rtol=0, atol=1e-4)
    if "confidence" in z:
        np.testing.assert_array_equal(host(o["confidence"]), z["confidence"])


@pytest.mark.parametrize("clip", [False, True])
def test_replay_offset_dump_bit_exact(clip, tmp_path):
    B, H, W, K = 2, 40, 56, 8
    s = synth(B, H, W, K, seed=31)
    cu = lambda x: torch.from_numpy(x).to(DEV)
    off_aff = cu(s["off_aff"])
    g = torch.tensor([4.0], device=DEV)
    with torch.no_grad():
        ref = propagate(cu(s["pred_init"]), cu(s["dep"]), cu(s["conf"]), off_aff[:, 2 * K:], off_aff[:, :2 * K], g,
                        prop_time=18, always_clip=clip)
        ref["gamma"] = g
        save_dump(str(tmp_path), ref)
        o = replay(load_dump(str(tmp_path)), s["pred_init"], s["dep"], s["conf"], prop_time=18, always_clip=clip,
                   device=DEV)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(o["pred_inter_tensor"]), host(ref["pred_inter_tensor"]))
    np.testing.assert_array_equal(host(o["pred"]), host(ref["pred"]))
    np.testing.assert_array_equal(host(o["confidence"]), host(ref["confidence"]))


def test_replay_1x17_fp16_dump(tmp_path, record_metric):
    B, H, W, K = 2, 48, 64, 16
    s = synth(B, H, W, K, seed=32)
    cu = lambda x: torch.from_numpy(x).to(DEV)
    off_aff = cu(s["off_aff"])
    g = torch.tensor([8.0], device=DEV)
    with torch.no_grad():
        ref = propagate(cu(s["pred_init"]), cu(s["dep"]), cu(s["conf"]), off_aff[:, 2 * K:], off_aff[:, :2 * K], g,
                        prop_time=36, kernel=(1, 17))
        ref["gamma"] = g
        save_dump(str(tmp_path), ref)
        d = load_dump(str(tmp_path), kernel=(1, 17))
        o32 = replay(d, s["pred_init"], s["dep"], s["conf"], prop_time=36, device=DEV)
        o16 = replay(d, s["pred_init"], s["dep"], s["conf"], prop_time=36, device=DEV, dtype=torch.float16)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(o32["pred"]), host(ref["pred"]))
    e = rmse(host(o16["pred"]), host(o32["pred"]))
    record_metric("replay_1x17_fp16_rmse", e)
    assert o16["pred"].dtype == torch.float16 and e <= 1e-2
