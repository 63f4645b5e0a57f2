"""Ablation of the head-epilogue kernel (NLSPN_HEADS_DBG bits: 1 no VALU chunks,
2 no MFMAs, 4 no staging) at NYU B=8: where the kernel's time goes.  Outputs are
garbage under any bit; timing only."""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the NLSPN_*_DBG switches exist only in the experiments build (make -C nlspn_eccv20_amd/csrc exp)
os.environ.setdefault("NLSPN_LIB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "nlspn_eccv20_amd", "lib", "exp", "libnlspn_hip_exp.so"))
from nlspn_eccv20_amd.heads import HeadWeights, head_epilogue  # noqa: E402
from tools.head_prof import timed  # noqa: E402


def main():
    dev = "cuda:0"
    B, H, W = (8, 228, 304) if len(sys.argv) < 2 else tuple(int(v) for v in sys.argv[1].split(","))
    g = torch.Generator(device=dev).manual_seed(0)
    src = [torch.rand((B, 64, H, W), device=dev, generator=g) for _ in range(4)]
    oa, idc, cfc = (nn.Conv2d(128, n, 3, padding=1).to(dev) for n in (24, 1, 1))
    hw = HeadWeights()
    res = {}
    with torch.no_grad():
        for dbg in (0, 1, 2, 3, 4, 5, 6, 7):
            os.environ["NLSPN_HEADS_DBG"] = str(dbg)
            res[dbg] = round(timed(lambda: head_epilogue(src[0], src[1], oa, src[2], idc, src[3], cfc, weights=hw)), 4)
    os.environ.pop("NLSPN_HEADS_DBG")
    print(json.dumps({"B": B, "H": H, "W": W, "ms_by_dbg": res,
                      "legend": "1 no VALU chunks, 2 no MFMAs, 4 no staging (global loads + LDS stores)"}))


if __name__ == "__main__":
    main()
