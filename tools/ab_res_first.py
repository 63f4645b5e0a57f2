"""Interleaved A/B of the resident section's first iteration: step 1 as its own launch
(default) vs inside the resident launches (NLSPN_RES_FIRST=1).  Both plans replay on
the same inputs in alternating rounds of 20, so box-to-box and drift noise cancel;
prints the median per-section time of each per config (JSON).
usage: python tools/ab_res_first.py [--rounds 15]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CONFIGS, make_inputs  # noqa: E402
from nlspn_eccv20_amd.propagation import PropagationPlan  # noqa: E402


def plan_for(inputs, cfg, first):
    if first:
        os.environ["NLSPN_RES_FIRST"] = "1"
    else:
        os.environ.pop("NLSPN_RES_FIRST", None)
    p = PropagationPlan(inputs["pred_init"], inputs["dep"], inputs["conf"], inputs["aff"], inputs["off"],
                        inputs["gamma"], prop_time=cfg["T"], kernel=cfg["kernel"])
    os.environ.pop("NLSPN_RES_FIRST", None)
    return p


def main(rounds=15, per=20):
    dev = torch.device("cuda", 0)
    out = {}
    for name in ("nyu", "kitti", "nyu_b1"):
        cfg = CONFIGS[name]
        inputs, _ = make_inputs(cfg, 0, dev)
        plans = {"step1_launch": plan_for(inputs, cfg, False), "first_in_resident": plan_for(inputs, cfg, True)}
        for p in plans.values():
            for _ in range(5):
                p.replay()
        torch.cuda.synchronize()
        times = {k: [] for k in plans}
        for r in range(rounds):
            for k in (list(plans) if r % 2 == 0 else list(plans)[::-1]):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(per):
                    plans[k].replay()
                torch.cuda.synchronize()
                times[k].append(1e6 * (time.perf_counter() - t0) / per)
        same = torch.equal(plans["step1_launch"].outputs["pred_inter"], plans["first_in_resident"].outputs["pred_inter"])
        for p in plans.values():
            p.check()
            p.close()
        med = {k: round(sorted(v)[len(v) // 2], 2) for k, v in times.items()}
        out[name] = {"us_per_section_median": med, "min": {k: round(min(v), 2) for k, v in times.items()},
                     "bit_identical": bool(same)}
    print(json.dumps(out))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    a = ap.parse_args()
    main(a.rounds)
