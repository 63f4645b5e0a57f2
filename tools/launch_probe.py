"""Per-step launch overhead probe: the whole propagation section (C2 by default) replayed
as one hipGraph (nlspn_plan_launch) vs issued as direct launches (nlspn_propagate), N
steps back to back on one stream, timed with events.  Prints one JSON line per mode."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd import _lib  # noqa: E402
from nlspn_eccv20_amd.propagation import PropagationPlan, _alloc_outputs, _propagate_args, _stream  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402


def main(B=8, H=228, W=304, T=18, steps=200):
    dev = torch.device("cuda", 0)
    s = synth(B, H, W, 8, seed=7240, density=500 / (H * W))
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    oa = t(s["off_aff"])
    ins = (t(s["pred_init"]), t(s["dep"]), t(s["conf"]), oa[:, 16:], oa[:, :16], torch.tensor([4.0], device=dev))
    plan = PropagationPlan(*ins, prop_time=T)
    outs = _alloc_outputs(ins[0], 8, T, True, True)
    args, _ = _propagate_args(*ins, (3, 3), T, "TGASS", True, False, outs)
    lib = _lib.get()
    st = _stream(dev)

    def direct():
        _lib.check(lib.nlspn_propagate(*args, st))

    for name, fn in (("graph", plan.replay), ("direct", direct), ("graph", plan.replay), ("direct", direct)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        print(json.dumps({"mode": name, "us_per_step": round(ms * 1e3, 2), "iters_per_s": round(T / ms * 1e3, 1)}),
              flush=True)
    same = torch.equal(plan.outputs["pred"], outs["pred"])
    print(json.dumps({"graph_equals_direct": bool(same)}))
    plan.close()


if __name__ == "__main__":
    main()
