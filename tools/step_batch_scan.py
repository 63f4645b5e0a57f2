"""Step-kernel time against the batch size at a fixed image shape (diagnostic): a
bandwidth-bound launch scales linearly with B; a sawtooth over B says the grid's last
round of workgroups (the tail) costs time.  Times prop_step with HIP-graph-free eager
launches, CUDA events over many reps; prints us per launch and per image.
usage: python tools/step_batch_scan.py [--kernel 1 17] [--dtype f16] [--H 228 --W 304]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd import prop_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", type=int, nargs=2, default=[1, 17])
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--H", type=int, default=228)
    ap.add_argument("--W", type=int, default=304)
    ap.add_argument("--batches", type=int, nargs="+", default=[4, 8, 10, 12, 14, 15, 16, 17, 18, 20, 24, 32])
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = "cuda:0"
    dt = torch.float16 if a.dtype == "f16" else torch.float32
    kh, kw = a.kernel
    K = kh * kw - 1
    g = torch.Generator(device="cpu").manual_seed(5)
    out = {"kernel": [kh, kw], "dtype": a.dtype, "H": a.H, "W": a.W, "rows": []}
    for B in a.batches:
        H, W = a.H, a.W
        p = torch.rand(B, 1, H, W, generator=g).to(dev, dt)
        conf = torch.rand(B, 1, H, W, generator=g).to(dev, dt)
        dep = torch.zeros(B, 1, H, W).to(dev, dt)
        aff = (torch.rand(B, K + 1, H, W, generator=g) / K).to(dev, dt)
        off = (2.0 * torch.randn(B, 2 * (K + 1), H, W, generator=g)).to(dev, dt)
        o = torch.empty_like(p)
        for _ in range(20):
            prop_step(p, conf, dep, aff, off, kernel=(kh, kw), out=o)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            prop_step(p, conf, dep, aff, off, kernel=(kh, kw), out=o)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        out["rows"].append({"B": B, "us": round(us, 2), "us_per_image": round(us / B, 3)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
