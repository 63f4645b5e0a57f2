"""Interleaved same-process A/B of two propagation plans that differ only in one
environment setting read at plan creation (default: NLSPN_RES_L2=0, every resident
hand-off write-through, vs same-XCD images' hand-offs kept in the XCD's L2).  Both
plans replay on the same inputs in alternating rounds of 20, so box-to-box and drift
noise cancel; prints the median per-section time of each per config (JSON).
usage: python tools/ab_env.py [--rounds 15] [--env NAME=VALUE] [--configs nyu,kitti]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CONFIGS, make_inputs  # noqa: E402
from nlspn_eccv20_amd.propagation import PropagationPlan  # noqa: E402


def plan_for(inputs, cfg, env):
    name, value = env.split("=", 1)
    old = os.environ.pop(name, None)
    if value:
        os.environ[name] = value
    try:
        return PropagationPlan(inputs["pred_init"], inputs["dep"], inputs["conf"], inputs["aff"], inputs["off"],
                               inputs["gamma"], prop_time=cfg["T"], kernel=cfg["kernel"])
    finally:
        os.environ.pop(name, None)
        if old is not None:
            os.environ[name] = old


def main(rounds=15, per=20, env="NLSPN_RES_L2=0", configs=("nyu", "kitti", "nyu_b1")):
    dev = torch.device("cuda", 0)
    out = {"B": env}
    name_ = env.split("=", 1)[0]
    for name in configs:
        cfg = CONFIGS[name]
        inputs, _ = make_inputs(cfg, 0, dev)
        plans = {"A_default": plan_for(inputs, cfg, name_ + "="), "B_" + env: plan_for(inputs, cfg, env)}
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
        pa, pb = plans.values()
        same = torch.equal(pa.outputs["pred_inter"], pb.outputs["pred_inter"])
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
    ap.add_argument("--env", default="NLSPN_RES_L2=0", help="the B plan's setting")
    ap.add_argument("--configs", default="nyu,kitti,nyu_b1")
    a = ap.parse_args()
    main(a.rounds, env=a.env, configs=tuple(a.configs.split(",")))
