"""Run-to-run spread of the section backward's gradients (float-atomic arrival order), resident
pass 1 against the step launches, on one shape (experiments build: NLSPN_LIB_PATH=lib/exp/...,
whose NLSPN_BWD_RESIDENT=0 keeps the steps).  Prints, per gradient, the largest elementwise
difference between repeated runs of each form and between the forms, absolute and relative to
the tensor's largest magnitude, and the relative L2 difference (JSON).
usage: python tools/bwd_determinism.py [--B 2 --H 40 --W 64 --T 6 --reps 4]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd.propagation import propagate  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=40)
    ap.add_argument("--W", type=int, default=64)
    ap.add_argument("--T", type=int, default=6)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    K = 8
    s = synth(a.B, a.H, a.W, K, seed=3)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    pi, dep, conf, oa = t(s["pred_init"]), t(s["dep"]), t(s["conf"]), t(s["off_aff"])
    g = torch.tensor([4.0], device=dev)

    def grads(resident):
        if resident:
            os.environ.pop("NLSPN_BWD_RESIDENT", None)
        else:
            os.environ["NLSPN_BWD_RESIDENT"] = "0"
        leaves = [x.detach().clone().requires_grad_(True) for x in (pi, conf, oa[:, 2 * K:], oa[:, :2 * K], g)]
        o = propagate(leaves[0], dep, leaves[1], leaves[2], leaves[3], leaves[4], prop_time=a.T)
        (o["pred"].square().sum() + o["pred_inter_tensor"][2].sum()).backward()
        torch.cuda.synchronize()
        return [x.grad.detach().clone() for x in leaves]

    names = ("pred_init", "confidence", "aff", "offset", "gamma")
    runs = {"resident": [grads(True) for _ in range(a.reps)], "steps": [grads(False) for _ in range(a.reps)]}
    os.environ.pop("NLSPN_BWD_RESIDENT", None)

    def cmp(x, y):
        d = (x - y).abs()
        m = max(float(y.abs().max()), 1e-30)
        return {"max_abs": float(d.max()), "max_abs_over_max": float(d.max()) / m,
                "max_rel_elem": float((d / y.abs().clamp_min(1e-30)).max()),
                "rel_l2": float((x - y).norm() / max(float(y.norm()), 1e-30)),
                "allclose_1e-5_1e-7": bool(torch.allclose(x, y, rtol=1e-5, atol=1e-7))}

    out = {"shape": [a.B, a.H, a.W, a.T], "reps": a.reps}
    for form, rs in runs.items():
        out[form + "_run_to_run"] = {n: [cmp(rs[i][k], rs[0][k]) for i in range(1, len(rs))][-1] for k, n in enumerate(names)}
    out["resident_vs_steps"] = {n: cmp(runs["resident"][0][k], runs["steps"][0][k]) for k, n in enumerate(names)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
