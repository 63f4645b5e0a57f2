"""Experiment harness for the resident kernel: time iterations 2..T (dispatch events)
with parts of the per-iteration work switched off (NLSPN_RES_DBG bits: 1 no wait,
2 no staging loads, 4 no taps), to see where an iteration's time goes.
Outputs of dbg != 0 runs are meaningless; only their timing is."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the NLSPN_*_DBG switches exist only in the experiments build (make -C nlspn_eccv20_amd/csrc exp)
os.environ.setdefault("NLSPN_LIB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "nlspn_eccv20_amd", "lib", "exp", "libnlspn_hip_exp.so"))
from nlspn_eccv20_amd import _lib  # noqa: E402
from nlspn_eccv20_amd.propagation import _alloc_outputs  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402


def run(B=8, H=228, W=304, T=18, reps=20, dbgs=(0, 1, 2, 4, 3, 6, 7), resident=("1",)):
    dev = torch.device("cuda", 0)
    s = synth(B, H, W, 8, seed=7240, off_sigma=2.0, density=500 / (H * W))
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    oa = t(s["off_aff"])
    pi, dep, conf = t(s["pred_init"]), t(s["dep"]), t(s["conf"])
    g = torch.tensor([4.0], device=dev)
    o = _alloc_outputs(pi, 8, T, True, True)
    lib = _lib.get()
    grid = ctypes.c_int()
    os.environ["NLSPN_RESIDENT"] = "1"
    lib.nlspn_resident_config(0, B, H, W, 3, 3, T, 1, ctypes.byref(grid), None, None)
    res = []
    for r in resident:
        for d in (dbgs if r == "1" else (0,)):
            os.environ["NLSPN_RESIDENT"] = r
            os.environ["NLSPN_RES_DBG"] = str(d)
            f, rest, rs = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
            _lib.check(lib.nlspn_time_propagate(
                0, pi.data_ptr(), dep.data_ptr(), conf.data_ptr(), oa[:, 16:].data_ptr(), oa.stride(0),
                oa.data_ptr(), oa.stride(0), g.data_ptr(), o["pred_inter"].data_ptr(), o["pred"].data_ptr(),
                o["aff"].data_ptr(), o["offset"].data_ptr(), o["confidence"].data_ptr(), o["workspace"].data_ptr(),
                B, H, W, 3, 3, T, 3, _lib.PRESERVE_INPUT, reps, torch.cuda.current_stream().cuda_stream,
                ctypes.byref(f), ctypes.byref(rest), ctypes.byref(rs)))
            row = {"resident": rs.value, "dbg": d, "first_us": round(f.value * 1e3, 2),
                   "rest_us": round(rest.value * 1e3, 2), "per_iter_us": round(rest.value * 1e3 / (T - 1), 3),
                   "abort": int(o["workspace"][grid.value].item()) if rs.value else 0}
            print(json.dumps(row), flush=True)
            res.append(row)
    os.environ.pop("NLSPN_RES_DBG", None)
    return res


if __name__ == "__main__":
    args = dict(a.split("=") for a in sys.argv[1:])
    run(B=int(args.get("B", 8)), H=int(args.get("H", 228)), W=int(args.get("W", 304)), T=int(args.get("T", 18)),
        resident=tuple(args.get("resident", "1,0").split(",")), reps=int(args.get("reps", 20)),
        dbgs=tuple(int(x) for x in args.get("dbgs", "0,1,2,4,3,6,7").split(",")))
