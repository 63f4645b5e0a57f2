"""Interleaved same-process A/B of backward variants that differ in environment settings read
per nlspn_propagate_backward call (experiments build: NLSPN_LIB_PATH=lib/exp/...): e.g.
NLSPN_BWD_RESIDENT=0 (pass 1 as per-iteration step launches), NLSPN_BWD_CW=0 (pass 2 stages
conf' every iteration), NLSPN_BWD_ONEPASS=1.  Times the propagation section's backward alone
(autograd.grad of pred with the forward's graph kept), in alternating rounds, on bench.py's
synthetic inputs; prints per-variant median ms per backward and per iteration (JSON).
usage: python tools/ab_bwd.py [--config nyu] [--rounds 9] [--per 10] NAME=ENV[,ENV...] ..."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CONFIGS, make_inputs  # noqa: E402
from nlspn_eccv20_amd.propagation import propagate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="nyu")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--T", type=int, default=0, help="prop_time (0: the config's)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = dict(CONFIGS[a.config])
    if a.T:
        cfg["T"] = a.T
    inputs, _ = make_inputs(cfg, 0, dev)
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    pi = inputs["pred_init"].detach().clone().requires_grad_(True)
    cf = inputs["conf"].detach().clone().requires_grad_(True)
    oa = torch.cat([inputs["off"], inputs["aff"]], 1).detach().requires_grad_(True)
    g = inputs["gamma"].detach().clone().requires_grad_(True)
    gp = torch.randn_like(pi)
    out = propagate(pi, inputs["dep"], cf, oa[:, 2 * K:], oa[:, :2 * K], g, prop_time=cfg["T"], kernel=cfg["kernel"])
    variants = {}
    for v in a.variants:
        name, _, envs = v.partition("=")
        variants[name] = [e.split(":", 1) if ":" in e else e.split("=", 1) for e in envs.split(",") if e]

    def run(envs):
        saved = {k: os.environ.get(k) for k, _ in envs}
        for k, val in envs:
            os.environ[k] = val
        try:
            return torch.autograd.grad(out["pred"], (pi, cf, oa, g), gp, retain_graph=True)
        finally:
            for k, old in saved.items():
                if old is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = old

    ref = None
    diffs = {}
    for name, envs in variants.items():
        for _ in range(3):
            gr = run(envs)
        torch.cuda.synchronize()
        gr = [x.detach().clone() for x in gr]
        if ref is None:
            ref = gr
        diffs[name] = max(float((x - y).norm() / max(y.norm(), 1e-30)) for x, y in zip(gr, ref))
    times = {n: [] for n in variants}
    for r in range(a.rounds):
        order = list(variants) if r % 2 == 0 else list(variants)[::-1]
        for name in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.per):
                run(variants[name])
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.per)
    res = {"config": a.config, "T": cfg["T"], "variants": a.variants, "rel_diff_vs_first": diffs}
    for name, t in times.items():
        t = sorted(t)
        res[name] = {"ms_bwd_median": round(t[len(t) // 2], 4), "ms_bwd_min": round(t[0], 4),
                     "us_per_iter_median": round(1e3 * t[len(t) // 2] / cfg["T"], 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
