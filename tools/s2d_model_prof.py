"""Times the model's whole S2D module (fused front + MIOpen 3x3 conv 17->32) at NYU size,
to see which kernel MIOpen picks for S2D.conv (run under rocprofv3 --kernel-trace --stats)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd.model import S2D  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = S2D().to(dev)
    dep = torch.rand((8, 1, 228, 304), device=dev) * 10
    dep = torch.where(torch.rand_like(dep) < 0.0072, dep, torch.zeros_like(dep))
    with torch.no_grad():
        for _ in range(20):
            m(dep)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            m(dep)
        e1.record()
        torch.cuda.synchronize()
    print(json.dumps({"s2d_module_us": round(e0.elapsed_time(e1) * 10, 2)}))


if __name__ == "__main__":
    main()
