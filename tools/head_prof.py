"""Time the reference's last head layers on the GPU (nlspnmodel.py:296-315): the three
`_concat` + 3x3 convs that produce pred_init (id_dec0, ReLU), off_aff (off_aff_dec0) and
confidence (cf_dec0, sigmoid), each from 64 decoder channels + the shared 64-channel fe1.
Prints one JSON line per config with the per-piece and total times (CUDA events, median
of 20 after 5 warm-ups).  Synthetic activations (ReLU-like, U(0,1)) and default-init weights.

usage: python tools/head_prof.py [--configs nyu,kitti]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"nyu": (8, 228, 304), "kitti": (4, 240, 1216)}


def timed(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="nyu,kitti")
    ap.add_argument("--K", type=int, default=8)
    args = ap.parse_args()
    dev = "cuda:0"
    torch.backends.cudnn.benchmark = True
    for name in args.configs.split(","):
        B, H, W = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        mk = lambda: torch.rand((B, 64, H, W), device=dev, generator=g)  # noqa: E731
        fe1, id_fd1, oa_fd1, cf_fd1 = mk(), mk(), mk(), mk()
        id_dec0 = nn.Conv2d(128, 1, 3, padding=1).to(dev)
        oa_dec0 = nn.Conv2d(128, 3 * args.K, 3, padding=1).to(dev)
        cf_dec0 = nn.Conv2d(128, 1, 3, padding=1).to(dev)

        def heads():
            with torch.no_grad():
                p = F.relu(id_dec0(torch.cat((id_fd1, fe1), 1)))
                oa = oa_dec0(torch.cat((oa_fd1, fe1), 1))
                c = torch.sigmoid(cf_dec0(torch.cat((cf_fd1, fe1), 1)))
            return p, oa, c

        cat = torch.cat((oa_fd1, fe1), 1)
        r = {"config": name, "B": B, "H": H, "W": W, "K": args.K}
        r["heads_total_ms"] = timed(heads)
        r["cat_ms"] = timed(lambda: torch.cat((oa_fd1, fe1), 1))
        with torch.no_grad():
            r["conv_off_aff_ms"] = timed(lambda: oa_dec0(cat))
            r["conv_1ch_ms"] = timed(lambda: cf_dec0(cat))
        macs = B * H * W * 128 * 9 * (3 * args.K + 2)
        try:
            from nlspn_eccv20_amd.heads import HeadWeights, head_epilogue
            hw = HeadWeights()
            with torch.no_grad():
                r["fused_ms"] = timed(lambda: head_epilogue(fe1, oa_fd1, oa_dec0, id_fd1, id_dec0, cf_fd1, cf_dec0,
                                                            weights=hw))
                f = head_epilogue(fe1, oa_fd1, oa_dec0, id_fd1, id_dec0, cf_fd1, cf_dec0, weights=hw)
                ref = heads()
            r["fused_max_abs_diff"] = max((a - b).abs().max().item() for a, b in zip(f, ref))
            r["speedup_vs_torch"] = round(r["heads_total_ms"] / r["fused_ms"], 2)
            # f32 matrix-core work actually issued: 32*MB rows x (2 sources x C x 9) per pixel
            mb = (3 * args.K + 2 + 31) // 32
            issued = B * H * W * 32 * mb * 2 * 64 * 9 + B * H * W * 2 * 64 * 9
            r["fused_tflops_useful"] = round(2 * macs / (r["fused_ms"] * 1e-3) / 1e12, 2)
            r["fused_tflops_issued"] = round(2 * issued / (r["fused_ms"] * 1e-3) / 1e12, 2)
            r["fused_frac_f32_peak_issued"] = round(r["fused_tflops_issued"] / 157.3, 3)
        except ImportError:
            pass
        r["tflops_convs_only"] = round(2 * macs / ((r["conv_off_aff_ms"] + 2 * r["conv_1ch_ms"]) * 1e-3) / 1e12, 2)
        r["tflops_total"] = round(2 * macs / (r["heads_total_ms"] * 1e-3) / 1e12, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
