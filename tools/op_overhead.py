"""Host cost per call of the propagation entry points at a launch-bound size (GRU mode
calls prop_step + affinity_normalization once per iteration): the Python host mirror
(ctypes into the C ABI) vs the torch operator layer (torch.ops.nlspn.*).  Reports the
mean wall time per call over many calls with a synchronize at the end (the GPU work is
tiny, so host dispatch dominates)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd import affinity_normalization, ops, prop_step  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402


def timeit(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    ops.load()
    dev = "cuda:0"
    s = synth(1, 16, 24, 8, seed=1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    oa = t(s["off_aff"])
    pi, dep, conf, aff, off, g = t(s["pred_init"]), t(s["dep"]), t(s["conf"]), oa[:, 16:], oa[:, :16], \
        torch.tensor([4.0], device=dev)
    an = affinity_normalization(aff, g)
    with torch.no_grad():
        r = {
            "prop_step_ctypes_us": timeit(lambda: prop_step(pi, conf, dep, an, off, offset_layout="raw")),
            "prop_step_torch_op_us": timeit(lambda: torch.ops.nlspn.prop_step(pi, conf, dep, an, off, 3, 3, True,
                                                                              True, False)),
            "affnorm_ctypes_us": timeit(lambda: affinity_normalization(aff, g)),
            "affnorm_torch_op_us": timeit(lambda: torch.ops.nlspn.affinity_normalization(aff, g, "TGASS")),
        }
    print(json.dumps({k: round(v, 2) for k, v in r.items()}))


if __name__ == "__main__":
    main()
