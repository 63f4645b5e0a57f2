"""Critical-path trace of the resident kernel (NLSPN_RES_DBG=8): thread 0 of every part
stamps s_memrealtime (100 MHz) at five points of each iteration — loop top (S0), before
staging (S1), after the staging barrier (S2: staging includes the spin on poisoned cells,
i.e. the hand-off latency plus the skew to the slowest producer), taps + stores issued
(S3), after the closing barrier (S4) — into the `pred` buffer.  Prints per-phase medians
(us) per image-group launch.  Builds with NLSPN_RES_WTRACE=1 add per-wave stamps.
usage: python tools/res_trace.py [--config nyu|kitti|nyu_b1|nyu_k16] [--bg IMAGES_PER_LAUNCH] [--out FILE]"""
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
from nlspn_eccv20_amd.propagation import _alloc_outputs, _propagate_args, _stream  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402


# B, H, W, density, tap geometry, T, storage
_NYU = 500 / (228 * 304)
CONFIGS = {"nyu": (8, 228, 304, _NYU, (3, 3), 18, torch.float32), "kitti": (4, 240, 1216, 0.05, (3, 3), 18, torch.float32),
           "nyu_b1": (1, 228, 304, _NYU, (3, 3), 18, torch.float32),
           "nyu_k16": (16, 228, 304, _NYU, (1, 17), 36, torch.float16)}


def main(config="nyu", reps=5, bg=None, out=None):
    B, H, W, density, kern, T, dt = CONFIGS[config]
    K = kern[0] * kern[1] - 1
    dev = torch.device("cuda", 0)
    s = synth(B, H, W, K, seed=7240, off_sigma=2.0, density=density)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev, dt)  # noqa: E731
    oa = t(s["off_aff"])
    ins = (t(s["pred_init"]), t(s["dep"]), t(s["conf"]), oa[:, 2 * K:], oa[:, :2 * K], torch.tensor([4.0], device=dev))
    lib = _lib.get()
    grid, blk = ctypes.c_int(), ctypes.c_int()
    os.environ["NLSPN_RESIDENT"] = "1"
    lib.nlspn_resident_config(0 if dt == torch.float32 else 1, B, H, W, kern[0], kern[1], T, 1, ctypes.byref(grid),
                              ctypes.byref(blk), None)
    G = grid.value  # parts of one image-group launch
    bg = bg or B    # images per launch (C3: 2)
    ng = (B + bg - 1) // bg
    g = G // bg
    os.environ["NLSPN_RES_DBG"] = "8"
    outs = _alloc_outputs(ins[0], K, T, True, True)
    args, _ = _propagate_args(*ins, kern, T, "TGASS", True, False, outs)
    for _ in range(reps):
        _lib.check(lib.nlspn_propagate(*args, _stream(dev)))
    torch.cuda.synchronize()
    os.environ.pop("NLSPN_RES_DBG")
    HW = H * W
    allst = outs["pred"].view(-1).view(torch.int64).cpu().numpy()
    ept = 8 // outs["pred"].element_size()  # pred elements per int64 stamp
    res = {}
    for grp in range(ng):
        o = grp * bg * HW // ept  # group k's stamps start at its own pred planes
        R = T + 1  # rows per part: the setup, then iteration t in row t + 1
        raw = allst[o: o + G * R * 5].reshape(G, R, 5)
        # with the prologue in the launch iteration 0 (the section's iteration 1) has a row;
        # after a step-1 launch the loop starts at t = 1 (row 1 stays empty)
        it0 = 1 if (raw[:, 1, 0] != 0).any() else 2
        st = raw.astype(np.float64) / 100.0  # us
        res[f"group{grp}"] = phases(st, it0)
        res[f"group{grp}"]["prologue_in_launch"] = it0 == 1
        # per-wave stamps (after every part's five): [part, row, wave, (taps+stores issued, drained)]
        if o + G * R * 29 <= allst.size:  # room for the per-wave stamps (small batches: not)
            wv = allst[o + G * R * 5: o + G * R * 29].reshape(G, R, 12, 2)
            s2 = raw[:, :, 2]
            if (wv[:, 0, :, 0] != 0).any():  # builds with per-wave stamps (NLSPN_RES_WTRACE=1)
                res[f"group{grp}"]["waves"] = waves(s2, wv, it0)
    line = json.dumps({"config": config, "parts_per_launch": G, "threads": blk.value, "images_per_launch": bg,
                       "groups": ng, **res})
    if out:  # the JSON alone (the runtime's stderr lines never land in the file)
        with open(out, "w") as f:
            f.write(line + "\n")
    print(line)


def phases(st, it0):
    st -= st[:, 0, 0].min()  # row 0: setup stamps (entry, invariants loaded, window zeroed, taps classified)
    su = st[:, 0, :]
    setup = {"entry_spread": su[:, 0].max() - su[:, 0].min(), "invariant_loads": np.median(su[:, 1] - su[:, 0]),
             "window": np.median(su[:, 2] - su[:, 1]), "classify": np.median(su[:, 3] - su[:, 2]),
             "geometry_to_loop": np.median(st[:, it0, 0] - su[:, 3]), "first_loop_top_max": st[:, it0, 0].max()}
    if (su[:, 4] > 0).any():  # the prologue's normalisation done (from entry), before the loads' barrier
        setup["normalised"] = np.median(su[:, 4] - su[:, 0])
    st = st[:, it0:, :]  # the launch's iterations (1..T with the prologue in it, else 2..T)
    ph = {"wait": st[:, :, 1] - st[:, :, 0], "stage": st[:, :, 2] - st[:, :, 1], "taps+store": st[:, :, 3] - st[:, :, 2],
          "drain+barrier": st[:, :, 4] - st[:, :, 3]}
    ph["loop"] = st[:, 1:, 0] - st[:, :-1, 4]
    out = {k: {"median": round(float(np.median(v)), 3), "p90": round(float(np.percentile(v, 90)), 3)}
           for k, v in ph.items()}
    span = st[:, -1, 4].max() - st[:, 0, 0].min()
    out["span_us"] = round(float(span), 2)
    out["per_iter_us"] = round(float(span) / st.shape[1], 3)
    out["setup"] = {k: round(float(v), 3) for k, v in setup.items()}
    return out


def waves(s2, wv, it0):
    """Per wave of a part: the median time (us) from the part's taps start (S2, after the
    staging barrier) to the wave's taps + stores issued and to its stores drained, over
    the launch's iterations after its first, and the SIMD the wave ran on (HW_ID bits 5:4,
    recorded at entry, row 0)."""
    hw = wv[:, 0, :, 0]
    nw = int(max(1, ((hw != 0).any(0)).sum()))
    rel = (wv[:, it0 + 1:, :nw, :].astype(np.float64) - s2[:, it0 + 1:, None, None].astype(np.float64)) / 100.0
    return {"simd": [int(np.bincount(((hw[:, w] >> 4) & 3).astype(np.int64), minlength=4).argmax()) for w in range(nw)],
            "issued": [round(float(np.median(rel[:, :, w, 0])), 3) for w in range(nw)],
            "drained": [round(float(np.median(rel[:, :, w, 1])), 3) for w in range(nw)]}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="nyu", choices=sorted(CONFIGS))
    ap.add_argument("--bg", type=int, default=None, help="images per resident launch (C3: 2)")
    ap.add_argument("--out", default=None, help="write the JSON line to this file")
    a = ap.parse_args()
    main(a.config, bg=a.bg, out=a.out)
