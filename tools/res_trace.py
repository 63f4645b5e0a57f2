"""Critical-path trace of the resident kernel (NLSPN_RES_DBG=8): thread 0 of every part
stamps s_memrealtime (100 MHz) at five points of each iteration — loop top (S0), after
the wait barrier (S1), after staging (S2), before the drain (S3), after the publish
barrier (S4) — into the `pred` buffer.  Prints per-phase medians (us) and the hand-off
latency: a part's wait exit minus the latest publish of its neighbour parts."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd import _lib  # noqa: E402
from nlspn_eccv20_amd.propagation import _alloc_outputs, _propagate_args, _stream  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402


def main(B=8, H=228, W=304, T=18, reps=5):
    dev = torch.device("cuda", 0)
    s = synth(B, H, W, 8, seed=7240, off_sigma=2.0, density=500 / (H * W))
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    oa = t(s["off_aff"])
    ins = (t(s["pred_init"]), t(s["dep"]), t(s["conf"]), oa[:, 16:], oa[:, :16], torch.tensor([4.0], device=dev))
    lib = _lib.get()
    grid = ctypes.c_int()
    os.environ["NLSPN_RESIDENT"] = "1"
    lib.nlspn_resident_config(0, B, H, W, 3, 3, T, 1, ctypes.byref(grid), None, None)
    G, g = grid.value, grid.value // B
    os.environ["NLSPN_RES_DBG"] = "8"
    outs = _alloc_outputs(ins[0], 8, T, True, True)
    args, _ = _propagate_args(*ins, (3, 3), T, "TGASS", True, False, outs)
    for _ in range(reps):
        _lib.check(lib.nlspn_propagate(*args, _stream(dev)))
    torch.cuda.synchronize()
    os.environ.pop("NLSPN_RES_DBG")
    st = outs["pred"].view(-1).view(torch.int64)[: G * T * 5].cpu().numpy().reshape(G, T, 5).astype(np.float64)
    st = st / 100.0  # us
    st -= st[:, 0, 0].min()  # row t = 0: setup stamps (entry, invariants loaded, window zeroed, taps classified)
    su = st[:, 0, :]
    setup = {"entry_spread": su[:, 0].max() - su[:, 0].min(), "invariant_loads": np.median(su[:, 1] - su[:, 0]),
             "window": np.median(su[:, 2] - su[:, 1]), "classify": np.median(su[:, 3] - su[:, 2]),
             "geometry_to_loop": np.median(st[:, 1, 0] - su[:, 3]), "first_loop_top_max": st[:, 1, 0].max()}
    st = st[:, 1:, :]  # iterations 2..T
    ph = {"wait": st[:, :, 1] - st[:, :, 0], "stage": st[:, :, 2] - st[:, :, 1], "taps+store": st[:, :, 3] - st[:, :, 2],
          "drain+barrier": st[:, :, 4] - st[:, :, 3]}
    ph["loop"] = st[:, 1:, 0] - st[:, :-1, 4]
    out = {k: {"median": round(float(np.median(v)), 3), "p90": round(float(np.percentile(v, 90)), 3)}
           for k, v in ph.items()}
    # hand-off latency: wait exit of part (j, b) at iteration t vs the latest publish of parts j-1..j+1 at t-1
    lat = []
    for blk in range(G):
        b, j = blk % B, blk // B
        nb = [jj * B + b for jj in (j - 1, j, j + 1) if 0 <= jj < g]
        for it in range(1, st.shape[1]):
            lat.append(st[blk, it, 1] - max(st[n, it - 1, 4] for n in nb))
    out["publish_to_wait_exit"] = {"median": round(float(np.median(lat)), 3), "p90": round(float(np.percentile(lat, 90)), 3)}
    span = st[:, -1, 4].max() - st[:, 0, 0].min()
    out["span_us"] = round(float(span), 2)
    out["per_iter_us"] = round(float(span) / st.shape[1], 3)
    out["setup"] = {k: round(float(v), 3) for k, v in setup.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
