"""Diagnose a resident-vs-step mismatch: per iteration plane, how many pixels differ and
where (rows, part, wave, lane), plus the control words.  Debug aid, not a test."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from nlspn_eccv20_amd import _lib, propagate  # noqa: E402
from test_gpu_resident import _inputs, resident_config  # noqa: E402


def main(B=8, H=228, W=304, T=18, sigma=2.0):
    inp, _ = _inputs(B, H, W, sigma=sigma)
    ok, grid, block, lds = resident_config(B, H, W, T=T)
    g = grid // B
    print(json.dumps({"resident": ok, "grid": grid, "block": block, "lds": lds, "parts_per_image": g}))
    os.environ["NLSPN_RESIDENT"] = "1"
    a = propagate(*inp, prop_time=T)
    os.environ["NLSPN_RESIDENT"] = "0"
    b = propagate(*inp, prop_time=T)
    torch.cuda.synchronize()
    Q = H * W // 4
    for t in range(T):
        pa, pb = a["pred_inter_tensor"][t, :, 0], b["pred_inter_tensor"][t, :, 0]
        d = (pa != pb)
        n = int(d.sum())
        row = {"t": t, "ndiff": n, "maxabs": float((pa - pb).abs().max())}
        if n:
            idx = d.nonzero()
            bb, yy, xx = idx[:, 0], idx[:, 1], idx[:, 2]
            p = yy * W + xx
            # part of a pixel: largest j with j*Q//g*4 <= p
            j = torch.zeros_like(p)
            for jj in range(g):
                j = torch.where(p >= (jj * Q // g) * 4, torch.full_like(p, jj), j)
            plo = (j * Q // g) * 4
            off = p - plo
            row.update({"imgs": sorted(set(bb.tolist()))[:16], "rows": [int(yy.min()), int(yy.max())],
                        "parts": sorted(set(j.tolist()))[:32],
                        "waves": sorted(set((off // 256).tolist()))[:16],
                        "lane_e": sorted(set(((off % 256) // 64).tolist())),
                        "first": [[int(v) for v in r] for r in idx[:8].tolist()]})
        print(json.dumps(row), flush=True)
    ws = a.get("workspace")
    print("ctl words: n/a (workspace internal to propagate())")


if __name__ == "__main__":
    kw = dict(arg.split("=") for arg in sys.argv[1:])
    main(**{k: (float(v) if k == "sigma" else int(v)) for k, v in kw.items()})
