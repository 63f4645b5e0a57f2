"""S2D front timing: the fused kernel (nlspn_s2d_pyramid) vs the reference's torch ops
(torch.where + six nn.MaxPool2d + two 1x1 conv/ReLU + cat, nlspnmodel.py:437-459) on
the same GPU, NYU (B=8, 228x304) and KITTI (B=4, 240x1216) sizes.  Roofline: 72
algorithmic bytes per pixel (dep read once, 17 output planes written)."""
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd.s2d import s2d_front  # noqa: E402


def torch_ops(dep, w1, b1, w2, b2, pools):
    pyr = []
    for pool in pools[:4]:
        z = -pool(torch.where(dep == 0, -999 * torch.ones_like(dep), -dep))
        pyr.append(torch.where(z == 999, torch.zeros_like(dep), z))
    for pool in pools[4:]:
        pyr.append(pool(dep))
    h = F.relu(F.conv2d(F.relu(F.conv2d(torch.cat(pyr, 1), w1, b1)), w2, b2))
    return torch.cat([h, dep], 1)


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    pools = [nn.MaxPool2d(s, 1, s // 2) for s in (3, 5, 7, 9, 11, 13)]
    for name, (B, H, W, dens) in {"nyu": (8, 228, 304, 500 / (228 * 304)), "kitti": (4, 240, 1216, 0.05)}.items():
        g = torch.Generator(device=dev).manual_seed(1)
        dep = torch.rand((B, 1, H, W), generator=g, device=dev) * 50
        dep = torch.where(torch.rand((B, 1, H, W), generator=g, device=dev) < dens, dep, torch.zeros_like(dep))
        w1, b1 = torch.randn(8, 6, 1, 1, device=dev), torch.randn(8, device=dev)
        w2, b2 = torch.randn(16, 8, 1, 1, device=dev), torch.randn(16, device=dev)
        with torch.no_grad():
            kt = timeit(lambda: s2d_front(dep, w1, b1, w2, b2))
            rt = timeit(lambda: torch_ops(dep, w1, b1, w2, b2, pools))
            same = torch.allclose(s2d_front(dep, w1, b1, w2, b2), torch_ops(dep, w1, b1, w2, b2, pools),
                                  rtol=1e-4, atol=1e-3)
        npx = B * H * W
        print(json.dumps({"config": name, "kernel_us": round(kt * 1e3, 2), "torch_ops_us": round(rt * 1e3, 2),
                          "speedup": round(rt / kt, 2), "achieved_gbs": round(72 * npx / (kt * 1e-3) / 1e9, 1),
                          "frac_of_8tbs": round(72 * npx / (kt * 1e-3) / 8e12, 3), "matches": bool(same)}))


if __name__ == "__main__":
    main()
