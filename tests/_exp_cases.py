"""GPU cases that need the EXPERIMENTS build of the library (lib/exp/libnlspn_hip_exp.so:
the NLSPN_RES_DBG switches exist only there).  Each runs in a child process started by
tests/test_gpu_resident.py with NLSPN_LIB_PATH pointing at that build, so the product
library of the test process never sees the switches.
usage: python tests/_exp_cases.py CASE [ARGS]  -> prints "ok ..." or raises."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd import PropagationPlan, _lib, propagate  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402

DEV = "cuda:0"


def _inputs(B, H, W, sigma=2.0, seed=3):
    s = synth(B, H, W, 8, seed=seed, off_sigma=sigma, density=0.05)
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(DEV)  # noqa: E731
    oa = cu(s["off_aff"])
    return (cu(s["pred_init"]), cu(s["dep"]), cu(s["conf"]), oa[:, 16:], oa[:, :16], torch.tensor([4.0], device=DEV))


def _dbg(v):
    if v is None:
        os.environ.pop("NLSPN_RES_DBG", None)
    else:
        os.environ["NLSPN_RES_DBG"] = str(v)


def abort(B, H, W, seed):
    """A resident launch that aborts (dbg 32: part 0 aborts at its first staging) sets the
    device's sticky status: check() raises RuntimeError, and the planes the aborted parts
    never wrote hold NaN — for every image group of a merged launch.  Afterwards the next
    call runs clean."""
    inp = _inputs(B, H, W, seed=seed)
    os.environ["NLSPN_RESIDENT"] = "1"
    _dbg(32)
    plan = PropagationPlan(*inp, prop_time=18)
    o = plan.replay()
    try:
        plan.check()
        raise AssertionError("the injected abort did not raise")
    except RuntimeError as e:
        assert "aborted" in str(e), e
    p = o["pred_inter_tensor"]
    assert torch.isnan(p[1:, 0]).any()  # the aborting part's own image
    if B == 4:  # KITTI: two groups of two in one merged launch; its quads of group 1 too
        assert torch.isnan(p[1:, 2]).any() and torch.isnan(o["pred"][2]).any()
    plan.close()
    _dbg(None)
    _lib.check_resident()  # the sticky word was cleared by the raise
    o = propagate(*inp, prop_time=18)
    torch.cuda.synchronize()
    _lib.check_resident()
    assert not torch.isnan(o["pred"]).any()
    print("ok abort", B, H, W)


def general_path(B, H, W, sigma):
    """The shape takes the resident kernel's fixed-halo window and its general path (taps
    outside the LDS window read global memory): switching that path off (dbg 64) changes
    the result, so the alternating-input test of this shape exercises its re-reads."""
    inp = _inputs(B, H, W, sigma=sigma, seed=31)
    os.environ["NLSPN_RESIDENT"] = "1"
    a = propagate(*inp, prop_time=18)["pred_inter_tensor"].clone()
    _dbg(64)
    b = propagate(*inp, prop_time=18)["pred_inter_tensor"].clone()
    _dbg(None)
    torch.cuda.synchronize()
    _lib.check_resident()
    assert not torch.equal(a, b), "the general path is not taken at this shape"
    print("ok general path taken", B, H, W, sigma)


def bwd_abort(B, H, W, seed):
    """The resident backward pass 1 aborting (NLSPN_BWD_RES_DBG=16: part 0 raises the abort at its
    first wait): the device's sticky status raises; image 0's gradients hold NaN (its parts fill
    the dL/dout, dL/dconf' and dL/df_0 cells they had not finished); the abort word is global, so
    parts of other images that spin long enough abort too — every image's gradients are either
    NaN-marked in all four tensors or equal to a clean call's, none silently wrong; the next call
    runs clean."""
    pi, dep, conf, aff, off, g = _inputs(B, H, W, seed=seed)

    def grads(dbg):
        if dbg is None:
            os.environ.pop("NLSPN_BWD_RES_DBG", None)
        else:
            os.environ["NLSPN_BWD_RES_DBG"] = str(dbg)
        leaves = [x.detach().clone().requires_grad_(True) for x in (pi, conf, aff, off, g)]
        o = propagate(leaves[0], dep, leaves[1], leaves[2], leaves[3], leaves[4], prop_time=18)
        o["pred"].sum().backward()
        torch.cuda.synchronize()
        os.environ.pop("NLSPN_BWD_RES_DBG", None)
        return [x.grad for x in leaves]

    ga = grads(16)
    try:
        _lib.check_resident()
        raise AssertionError("the injected backward abort did not raise")
    except RuntimeError as e:
        assert "aborted" in str(e), e
    gc = grads(None)
    _lib.check_resident()
    assert all(torch.isfinite(x).all() for x in gc)
    rel = lambda x, y: float((x - y).norm() / y.norm())  # noqa: E731
    aborted = []
    for i in range(B):
        nan = [bool(torch.isnan(x[i]).any()) for x in ga[:4]]
        if i == 0 or any(nan):
            assert all(nan), (i, nan)  # every gradient of an aborted image is marked
            aborted.append(i)
        else:
            for x, y in zip(ga[:4], gc[:4]):
                assert rel(x[i], y[i]) < 1e-6, (i, rel(x[i], y[i]))
    print("ok bwd_abort", B, H, W, "aborted images", aborted)


if __name__ == "__main__":
    assert "exp" in _lib.LIB_PATH, f"needs the experiments build, got {_lib.LIB_PATH}"
    case, args = sys.argv[1], [float(x) if "." in x else int(x) for x in sys.argv[2:]]
    {"abort": abort, "general_path": general_path, "bwd_abort": bwd_abort}[case](*args)
