"""GPU: the resident propagation kernel (the prologue and iterations 1..T in one launch
per image group — or iterations 2..T after a step-1 launch, NLSPN_RES_FIRST=0 — invariant
planes on chip, poisoned-plane hand-offs) against the per-iteration launches and the oracle.

Bar: BIT-EXACT against step 1 + the T-1 per-iteration launches (all forms issue the
same IEEE sequence per pixel; only the schedule and the hand-off differ), every one
of the T pred_inter planes and the prologue's outputs, and no abort raised.  Exercised where hand-offs are most
fragile: long-range offsets (dependency ranges over many parts, taps beyond the
LDS window), tiny parts, repeated graph replays (a stale read shows up as a
replay that differs), fp16 storage, and every flag combination.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import PropagationPlan, _lib, propagate
from nlspn_eccv20_amd.synthetic import rmse, synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def cu(x, dtype=torch.float32):
    return None if x is None else torch.from_numpy(np.ascontiguousarray(x)).to(DEV, dtype)


def resident_config(B, H, W, dtype=0, conf=True, T=18, kernel=(3, 3)):
    g, b, l = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    ok = _lib.get().nlspn_resident_config(dtype, B, H, W, kernel[0], kernel[1], T, int(conf), ctypes.byref(g), ctypes.byref(b),
                                          ctypes.byref(l))
    return bool(ok), g.value, b.value, l.value


class _env:
    def __init__(self, value, name="NLSPN_RESIDENT"):
        self.value, self.name = value, name

    def __enter__(self):
        self.old = os.environ.get(self.name)
        os.environ[self.name] = self.value

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop(self.name, None)
        else:
            os.environ[self.name] = self.old


def _inputs(B, H, W, sigma=2.0, seed=3, dtype=torch.float32, conf=True, density=0.05, K=8):
    s = synth(B, H, W, K, seed=seed, off_sigma=sigma, density=density)
    oa = cu(s["off_aff"], dtype)
    return (cu(s["pred_init"], dtype), cu(s["dep"], dtype), cu(s["conf"], dtype) if conf else None,
            oa[:, 2 * K:], oa[:, :2 * K], torch.tensor([4.0], device=DEV)), s


def _nan_equal(x, y):
    """Equal NaN positions and bit-equal values elsewhere (a NaN's payload depends on which
    operation made it, not on the propagation it encodes)."""
    return torch.equal(torch.isnan(x), torch.isnan(y)) and _bits_equal(x.nan_to_num(7.0), y.nan_to_num(7.0))


def _both(inp, T=18, nan_ok=False, **kw):
    """(resident, steps): the default resident form (since round 5 the prologue and
    iteration 1 inside the resident launches, no step-1 launch), checked here against the
    resident form behind a step-1 launch (NLSPN_RES_FIRST=0), with every hand-off
    write-through (NLSPN_RES_L2=0: no line of any image kept in an XCD's L2), and the step
    form — every pred_inter plane, pred and the prologue's output-dict tensors.
    nan_ok: NaN results compare by position (_nan_equal)."""
    with _env("1"):
        a = propagate(*inp, prop_time=T, **kw)
        with _env("0", "NLSPN_RES_L2"):
            c = propagate(*inp, prop_time=T, **kw)
        with _env("0", "NLSPN_RES_FIRST"):
            f = propagate(*inp, prop_time=T, **kw)
        with _env("0", "NLSPN_RES_SPLIT"):  # (small parts: one thread per quad instead of four)
            g = propagate(*inp, prop_time=T, **kw)
        with _env("2", "NLSPN_RES_SPLIT"):  # (two threads per quad)
            h = propagate(*inp, prop_time=T, **kw)
    with _env("0"):
        b = propagate(*inp, prop_time=T, **kw)
    torch.cuda.synchronize()
    for k in ("aff", "offset", "confidence"):  # the prologue's output-dict tensors
        if a[k] is not None or b[k] is not None:
            assert _bits_equal(a[k], b[k]), k
            assert _bits_equal(c[k], b[k]), k
            assert _bits_equal(f[k], b[k]), k
    eq = _nan_equal if nan_ok else _bits_equal
    assert eq(a["pred_inter_tensor"], c["pred_inter_tensor"]), "resident forms differ"
    assert eq(a["pred"], c["pred"])
    assert eq(a["pred_inter_tensor"], f["pred_inter_tensor"]), "prologue in the launch and step 1 differ"
    assert eq(a["pred"], f["pred"])
    assert eq(a["pred_inter_tensor"], g["pred_inter_tensor"]), "split-quad and quad-per-thread builds differ"
    assert eq(a["pred"], g["pred"])
    assert eq(a["pred_inter_tensor"], h["pred_inter_tensor"]), "four- and two-thread split-quad builds differ"
    assert eq(a["pred"], h["pred"])
    return a, b


def _bits_equal(x, y):
    """Bit-for-bit equality (NaN offsets pass through unchanged, and NaN != NaN)."""
    it = torch.int32 if x.dtype == torch.float32 else torch.int16
    return x.dtype == y.dtype and torch.equal(x.view(it), y.view(it))


def test_resident_engaged_at_c2():
    with _env("1"):
        ok, grid, block, lds = resident_config(8, 228, 304)
        assert ok and grid == 256 and block == 576 and lds > 80 * 1024
        ok, grid, block, lds = resident_config(4, 240, 1216)  # C3: two groups of 2 images x 128 parts
        assert ok and grid == 256 and block == 576 and lds > 80 * 1024
        assert resident_config(8, 228, 304, dtype=1)[2] == 576  # fp16
        assert not resident_config(8, 228, 302)[0]       # W % 4 != 0
        ok, grid, block, lds = resident_config(1, 228, 304)  # C1: one image in 13 x 19 parts of 72 quads,
        assert ok and grid == 247 and block == 320          # four threads per quad (a split-quad build)
        with _env("2", "NLSPN_RES_SPLIT"):
            assert resident_config(1, 228, 304)[2] == 192   # two threads per quad
        with _env("0", "NLSPN_RES_SPLIT"):
            assert resident_config(1, 228, 304)[2] == 128   # a thread per quad
        # C5 (1x17, fp16, 16 images): four groups of four images in 9 x 7 parts of 286 quads, two
        # threads per quad (the 576-thread build; not three groups of five and one of one)
        ok, grid, block, lds = resident_config(16, 228, 304, dtype=1, T=36, kernel=(1, 17))
        assert ok and grid == 4 * 63 and block == 576


@pytest.mark.parametrize("B,H,W,sigma,dtype,conf,kw", [
    (8, 228, 304, 2.0, torch.float32, True, {}),                        # C2
    (8, 228, 304, 2.0, torch.float32, True, {"always_clip": True}),
    (8, 228, 304, 2.0, torch.float32, False, {"preserve_input": False}),
    (8, 228, 304, 2.0, torch.float16, True, {}),                        # fp16 storage
    (8, 228, 304, 12.0, torch.float32, True, {"always_clip": True}),    # C2 parts, fixed halo: the general path
    (4, 96, 128, 12.0, torch.float32, True, {}),                        # taps beyond the halo
    (2, 64, 96, 60.0, torch.float32, True, {"affinity": "TC"}),         # mostly out of image, long ranges
    (1, 24, 32, 2.0, torch.float32, True, {}),                          # 3 tiny parts
    (32, 40, 64, 2.0, torch.float32, True, {"affinity": "ASS"}),        # many images, 8 parts each
    (3, 50, 100, 4.0, torch.float32, True, {"affinity": "AS"}),         # B not dividing the CU count
    (4, 240, 1216, 2.0, torch.float32, True, {}),                       # C3: two image groups
    (5, 240, 1216, 3.0, torch.float32, True, {"always_clip": True}),    # groups of 2, 2, 1
    (4, 240, 1216, 2.0, torch.float16, True, {}),                       # C3 shape, fp16 storage
    (2, 120, 2048, 12.0, torch.float32, True, {}),                      # wide image, taps beyond the halo
])
def test_resident_bitexact_vs_steps(B, H, W, sigma, dtype, conf, kw):
    with _env("1"):
        assert resident_config(B, H, W, 0 if dtype == torch.float32 else 1, conf)[0]
    inp, _ = _inputs(B, H, W, sigma=sigma, dtype=dtype, conf=conf)
    a, b = _both(inp, **kw)
    assert torch.equal(a["pred_inter_tensor"], b["pred_inter_tensor"])
    assert torch.equal(a["pred"], b["pred"])


@pytest.mark.parametrize("B,H,W,sigma,dtype,kernel,T", [
    (16, 228, 304, 2.0, torch.float16, (1, 17), 36),   # C5: four image groups of four, one launch
    (16, 228, 304, 2.0, torch.float32, (1, 17), 36),   # C5 shape, fp32 storage
    (4, 96, 128, 3.0, torch.float32, (1, 17), 18),
    (3, 64, 96, 12.0, torch.float16, (1, 17), 18),     # taps beyond the halo (general path)
    (1, 24, 32, 2.0, torch.float16, (1, 17), 5),       # tiny parts
    (2, 64, 96, 2.0, torch.float32, (5, 5), 18),
    (2, 60, 128, 6.0, torch.float16, (5, 5), 18),
    (8, 228, 304, 2.0, torch.float16, (5, 5), 6),      # one launch per image group (no GROUPS build)
])
def test_resident_wide_geometry_bitexact(B, H, W, sigma, dtype, kernel, T):
    """The resident kernel's 1x17 (two pixels per thread) and 5x5 (a pixel per thread)
    builds: bit-exact against the step launches, every plane, both resident forms."""
    K = kernel[0] * kernel[1] - 1
    with _env("1"):
        assert resident_config(B, H, W, 0 if dtype == torch.float32 else 1, True, T, kernel)[0]
    inp, _ = _inputs(B, H, W, sigma=sigma, dtype=dtype, K=K)
    a, b = _both(inp, T=T, kernel=kernel)
    assert torch.equal(a["pred_inter_tensor"], b["pred_inter_tensor"])
    assert torch.equal(a["pred"], b["pred"])


@pytest.mark.parametrize("B,H,W,sigma,dtype,kw,block", [
    (1, 228, 304, 2.0, torch.float16, {}, 320),                         # C1 shape, fp16 storage
    (1, 228, 304, 12.0, torch.float32, {"always_clip": True}, 320),     # fixed halo: the general path
    (1, 228, 304, 2.0, torch.float32, {"preserve_input": False}, 320),
    (2, 100, 120, 3.0, torch.float32, {"affinity": "TC"}, 320),
    (1, 37, 52, 60.0, torch.float32, {}, None),                          # tiny, long ranges
])
def test_split_quad_builds_bitexact(B, H, W, sigma, dtype, kw, block):
    """Small parts split their quads over four (or two) threads: bit-exact against the step
    launches and the quad-per-thread build (_both), general path and fp16 included."""
    with _env("1"):
        ok, _, blk, _ = resident_config(B, H, W, 0 if dtype == torch.float32 else 1)
        assert ok and (block is None or blk == block)
    inp, _ = _inputs(B, H, W, sigma=sigma, dtype=dtype)
    a, b = _both(inp, **kw)
    assert torch.equal(a["pred_inter_tensor"], b["pred_inter_tensor"])
    assert torch.equal(a["pred"], b["pred"])


@pytest.mark.parametrize("T", [2, 3, 36])
def test_resident_bitexact_short_and_long(T):
    inp, _ = _inputs(4, 64, 128, sigma=3.0)
    a, b = _both(inp, T=T)
    assert torch.equal(a["pred_inter_tensor"], b["pred_inter_tensor"])
    assert torch.equal(a["pred"], b["pred"])


def test_plan_direct_equals_graph():
    """The resident plan re-issues its two launches directly; forcing the hipGraph
    replay gives the same bits."""
    inp, _ = _inputs(8, 228, 304, sigma=2.0, seed=5)
    outs = []
    for graph in ("0", "1"):
        os.environ["NLSPN_PLAN_GRAPH"] = graph
        try:
            with _env("1"):
                plan = PropagationPlan(*inp, prop_time=18)
                plan.replay()
                plan.replay()
                torch.cuda.synchronize()
                outs.append(plan.outputs["pred_inter"].clone())
                plan.close()
        finally:
            os.environ.pop("NLSPN_PLAN_GRAPH", None)
    assert torch.equal(outs[0], outs[1])


def test_resident_nonfinite_offsets():
    inp, _ = _inputs(2, 64, 128)
    off = inp[4].clone()
    off[0, 3, 5, 7] = float("nan")
    off[1, 0, 10, 11] = float("inf")
    off[1, 9, 40, 12] = -1e30
    inp = inp[:4] + (off, inp[5])
    a, b = _both(inp)
    assert torch.equal(a["pred_inter_tensor"].nan_to_num(7.0), b["pred_inter_tensor"].nan_to_num(7.0))


@pytest.mark.parametrize("cell", [(30, 50), (0, 127), (63, 0), (31, 72)])
def test_resident_reference_tap_nonfinite_neighbour(oracle, cell):
    """An inf depth makes its LEFT and UPPER neighbours NaN through their zero-offset
    reference tap: the reference samples all four corners of the integer point with
    weights (1, 0, 0, 0) (modulated_deform_im2col_cuda.cuh:37-52), 0 * inf = NaN.  The
    resident kernel (iterations 2..T) and the step launches both take the four-corner
    form when the window holds a non-finite f: the same NaN pattern as the oracle, and
    bit-equal values elsewhere.  Cells: interior, image corners / edges, a part seam."""
    inp, s = _inputs(2, 64, 128, seed=21)
    y, x = cell
    pi, dep = inp[0].clone(), inp[1].clone()
    pi[1, 0, y, x] = float("inf")
    dep[1, 0, max(y - 1, 0):y + 2, max(x - 1, 0):x + 2] = 0.0  # no preserve blend over the probe
    inp = (pi, dep) + inp[2:]
    T = 3
    a, b = _both(inp, T=T, nan_ok=True)
    for k in ("pred_inter_tensor", "pred"):
        assert _nan_equal(a[k], b[k]), k
    pin, dp = s["pred_init"].copy(), s["dep"].copy()
    pin[1, 0, y, x] = np.inf
    dp[1, 0, max(y - 1, 0):y + 2, max(x - 1, 0):x + 2] = 0.0
    e = oracle.propagate(pin, dp, s["conf"], s["off_aff"][:, 16:], s["off_aff"][:, :16], 4.0, prop_time=T)
    got = a["pred_inter_tensor"].cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(e["pred_inter"]))
    # iteration 1 (step 1): the inf cell's left / upper neighbours are NaN (their own taps
    # may hit it too; the reference tap alone guarantees it)
    for ny, nx in ((y, x - 1), (y - 1, x), (y - 1, x - 1)):
        if ny >= 0 and nx >= 0:
            assert np.isnan(got[0, 1, 0, ny, nx]), (ny, nx)
    assert np.isnan(got[1]).sum() > np.isnan(got[0]).sum()  # spreads in the resident iterations


def test_resident_replays_stable_and_no_abort():
    """A hand-off that could read a stale plane shows up as a replay that differs."""
    inp, _ = _inputs(8, 228, 304, sigma=3.0, seed=11)
    with _env("0"):
        ref = propagate(*inp, prop_time=18)["pred_inter_tensor"].clone()
    with _env("1"):
        plan = PropagationPlan(*inp, prop_time=18)
        for i in range(30):
            o = plan.replay()
            if i % 5 == 0:  # uneven load between replays: a busy stream beside the plan
                x = torch.randn(4096, 4096, device=DEV)
                _ = x @ x
            torch.cuda.synchronize()
            assert torch.equal(o["pred_inter_tensor"], ref), f"replay {i} differs"
            grid = resident_config(8, 228, 304)[1]
            assert grid > 0
            assert int(plan.outputs["workspace"][0].item()) == 0, "resident kernel aborted"
        plan.close()


@pytest.mark.parametrize("B,H,W,l2,dtype,sigma,kernel,T", [
    (8, 228, 304, "1", torch.float32, 3.0, (3, 3), 18), (8, 228, 304, "0", torch.float32, 3.0, (3, 3), 18),
    (4, 240, 1216, "1", torch.float32, 3.0, (3, 3), 18), (1, 228, 304, "1", torch.float32, 3.0, (3, 3), 18),
    (8, 228, 304, "1", torch.float16, 3.0, (3, 3), 18),
    (4, 240, 1216, "1", torch.float16, 3.0, (3, 3), 18),                 # C3 shape, fp16 lines (16 quads)
    (16, 228, 304, "1", torch.float16, 3.0, (1, 17), 36),                # C5: four groups, images over two XCDs
    (16, 228, 304, "0", torch.float16, 3.0, (1, 17), 36),
    (8, 228, 304, "1", torch.float32, 12.0, (3, 3), 18), (2, 120, 2048, "1", torch.float32, 12.0, (3, 3), 18)])
def test_resident_alternating_inputs_no_stale_reads(B, H, W, l2, dtype, sigma, kernel, T):
    """Replays over in-place refilled inputs that alternate between two data sets: every
    plane a hand-off reads was last written with the OTHER set's values, so a consumer that
    took a previous call's cell instead of waiting out the poison (nlspn_resident.h) changes
    the result.  Long-range offsets (sigma 3), per-line hand-offs (lines no part on another
    XCC reads kept in L2, the rest write-through) and every line write-through (l2 "0"), the
    two-group merged launch (KITTI B=4), one image over 247 parts, fp16 storage, C5's four
    image groups of 1x17 taps; and two fixed-halo shapes at sigma 12 whose far taps take the
    general path (global re-reads of the same cells every iteration, whole-image published
    windows; test_general_path_taken_at_fixed_halo_shapes)."""
    K = kernel[0] * kernel[1] - 1
    ia, _ = _inputs(B, H, W, sigma=sigma, seed=31, dtype=dtype, K=K)
    ib, _ = _inputs(B, H, W, sigma=sigma, seed=32, dtype=dtype, K=K)
    with _env("0"):
        ra = propagate(*ia, prop_time=T, kernel=kernel)["pred_inter_tensor"].clone()
        rb = propagate(*ib, prop_time=T, kernel=kernel)["pred_inter_tensor"].clone()
    buf = [None if x is None else x.clone() for x in ia]
    with _env("1"), _env(l2, "NLSPN_RES_L2"):
        plan = PropagationPlan(*buf, prop_time=T, kernel=kernel)
        for i in range(12):
            src, ref = (ia, ra) if i % 2 == 0 else (ib, rb)
            for d, x in zip(buf, src):
                if d is not None:
                    d.copy_(x)
            o = plan.replay()
            torch.cuda.synchronize()
            assert _bits_equal(o["pred_inter_tensor"], ref), f"replay {i}"
        plan.check()
        plan.close()


def test_resident_vs_oracle_c2(oracle):
    inp, s = _inputs(8, 228, 304, seed=7240)
    with _env("1"):
        o = propagate(*inp, prop_time=18)
    e = oracle.propagate(s["pred_init"], s["dep"], s["conf"], s["off_aff"][:, 16:], s["off_aff"][:, :16], 4.0)
    assert rmse(o["pred"].cpu().numpy(), e["pred"]) <= 1e-4


def test_time_propagate_reports_resident():
    inp, _ = _inputs(8, 228, 304)
    pi, dep, conf, aff, off, g = inp

    def timed(o):
        first, rest, res = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
        _lib.check(_lib.get().nlspn_time_propagate(
            0, pi.data_ptr(), dep.data_ptr(), conf.data_ptr(), aff.data_ptr(), aff.stride(0), off.data_ptr(),
            off.stride(0), g.data_ptr(), o["pred_inter"].data_ptr(), o["pred"].data_ptr(), o["aff"].data_ptr(),
            o["offset"].data_ptr(), o["confidence"].data_ptr(), o["workspace"].data_ptr(), 8, 228, 304, 3, 3, 18, 3,
            _lib.PRESERVE_INPUT, 3, torch.cuda.current_stream().cuda_stream, ctypes.byref(first),
            ctypes.byref(rest), ctypes.byref(res)))
        return first.value, rest.value, res.value

    with _env("1"):
        plan = PropagationPlan(*inp, prop_time=18)
        first, rest, res = timed(plan.outputs)
        # one resident launch (one image group) with the prologue inside (0x100): no step 1
        assert res == 0x101 and first >= 0 and first < 0.01 and rest > 0
        with _env("0", "NLSPN_RES_FIRST"):
            first, rest, res = timed(plan.outputs)
        assert res == 1 and first > 0 and rest > 0  # behind step 1
        plan.close()


def test_c3_resident_vs_oracle_and_replays(oracle):
    """C3 (KITTI B=4) runs iterations 2..T as two image groups of two images each, in
    turn inside one resident launch (a part sets up group 2 while others finish group 1):
    against the oracle at the north-star bar, and stable over plan replays."""
    inp, s = _inputs(4, 240, 1216, seed=7240)
    with _env("1"):
        plan = PropagationPlan(*inp, prop_time=18)
        ref = None
        for i in range(6):
            o = plan.replay()
            torch.cuda.synchronize()
            if ref is None:
                ref = o["pred_inter_tensor"].clone()
            assert torch.equal(o["pred_inter_tensor"], ref), f"replay {i} differs"
        plan.check()
        e = oracle.propagate(s["pred_init"], s["dep"], s["conf"], s["off_aff"][:, 16:], s["off_aff"][:, :16], 4.0)
        assert rmse(o["pred"].cpu().numpy(), e["pred"]) <= 1e-4
        plan.close()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_merged_groups_and_partial_group_bit_exact(dtype):
    """KITTI B=5: image groups of two, so the two full groups run in turn inside ONE
    launch (the GROUPS build) and the partial fifth image in a launch of its own —
    bit-exact against the step launches, against iteration 1 inside the launches, and
    against one launch per group (NLSPN_RES_MERGE=0)."""
    inp, _ = _inputs(5, 240, 1216, seed=11, dtype=dtype)
    a, b = _both(inp)
    assert _bits_equal(a["pred_inter_tensor"], b["pred_inter_tensor"])
    assert _bits_equal(a["pred"], b["pred"])
    with _env("1"), _env("0", "NLSPN_RES_MERGE"):
        c = propagate(*inp, prop_time=18)
    torch.cuda.synchronize()
    assert _bits_equal(a["pred_inter_tensor"], c["pred_inter_tensor"])
    # every hand-off write-through (no same-XCD L2 mode): the launch-tagged XCC ids of the
    # later launches (the partial group; each unmerged group) must not change the result
    for merge in ("1", "0"):
        with _env("1"), _env("0", "NLSPN_RES_L2"), _env(merge, "NLSPN_RES_MERGE"):
            d = propagate(*inp, prop_time=18)
        torch.cuda.synchronize()
        assert _bits_equal(a["pred_inter_tensor"], d["pred_inter_tensor"]), merge
    _lib.check_resident()


def test_two_plans_on_two_streams_bit_exact():
    """Two resident plans replayed concurrently on two streams of one device: the
    library serialises resident launches across streams (co-residency), so every
    replay is bit-exact and nothing aborts (never silent garbage)."""
    inp_a, _ = _inputs(8, 228, 304, seed=21)
    inp_b, _ = _inputs(8, 228, 304, seed=22)
    with _env("1"):
        ref_a = propagate(*inp_a, prop_time=18)["pred_inter_tensor"].clone()
        ref_b = propagate(*inp_b, prop_time=18)["pred_inter_tensor"].clone()
        torch.cuda.synchronize()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        with torch.cuda.stream(s1):
            pa = PropagationPlan(*inp_a, prop_time=18)
        with torch.cuda.stream(s2):
            pb = PropagationPlan(*inp_b, prop_time=18)
        torch.cuda.synchronize()
        for i in range(12):
            with torch.cuda.stream(s1):
                oa = pa.replay()
            with torch.cuda.stream(s2):
                ob = pb.replay()
            if i % 4 == 3:
                torch.cuda.synchronize()
                assert torch.equal(oa["pred_inter_tensor"], ref_a), f"plan A replay {i}"
                assert torch.equal(ob["pred_inter_tensor"], ref_b), f"plan B replay {i}"
        pa.check()
        pb.check()
        pa.close()
        pb.close()


def _exp_case(*args):
    """Runs a case of tests/_exp_cases.py in a child process on the EXPERIMENTS build of the
    library (the NLSPN_RES_DBG switches exist only there; the product library ignores them)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "nlspn_eccv20_amd", "lib", "exp", "libnlspn_hip_exp.so")
    assert os.path.exists(lib), "experiments build missing: make -C nlspn_eccv20_amd/csrc exp"
    env = dict(os.environ, NLSPN_LIB_PATH=lib)
    env.pop("NLSPN_RES_DBG", None)
    out = subprocess.run([sys.executable, os.path.join(root, "tests", "_exp_cases.py")] + [str(a) for a in args],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0 and "ok" in out.stdout, (out.stdout[-2000:], out.stderr[-3000:])


@pytest.mark.parametrize("B,H,W,seed", [(8, 228, 304, 5), (4, 240, 1216, 12)])
def test_aborted_launch_raises_and_poisons(B, H, W, seed):
    """A resident launch that aborts (experiments build, NLSPN_RES_DBG=32: part 0 aborts)
    sets the device's sticky status: check() raises RuntimeError and the planes the
    aborted parts never wrote hold NaN, not plausible depths — in a one-group launch (C2)
    and in a merged two-group launch (KITTI B=4), every group.  The next call runs clean."""
    _exp_case("abort", B, H, W, seed)


def test_product_library_ignores_experiment_switches():
    """The product library reads no NLSPN_RES_DBG: with the abort bit set in the
    environment a propagation is bit-exact and nothing aborts."""
    inp, _ = _inputs(8, 228, 304, seed=5)
    with _env("1"):
        ref = propagate(*inp, prop_time=18)["pred_inter_tensor"].clone()
        with _env("32", "NLSPN_RES_DBG"):
            o = propagate(*inp, prop_time=18)["pred_inter_tensor"]
    torch.cuda.synchronize()
    _lib.check_resident()
    assert torch.equal(o, ref)


@pytest.mark.parametrize("B,H,W,sigma", [(8, 228, 304, 12.0), (2, 120, 2048, 12.0)])
def test_general_path_taken_at_fixed_halo_shapes(B, H, W, sigma):
    """The fixed-halo shapes of the alternating-input test do take the general path (its
    results change when the experiments build switches that path off)."""
    _exp_case("general_path", B, H, W, sigma)


def test_plan_first_in_fresh_process():
    """A PropagationPlan created before any other library call (as bench.py does) in a
    fresh process: the library's one-time per-device setup must not run inside the
    plan's stream capture."""
    import subprocess
    import sys
    code = ("import sys, torch; sys.path.insert(0, %r)\n"
            "from nlspn_eccv20_amd import PropagationPlan\n"
            "d = 'cuda:0'; B, H, W, K = 8, 228, 304, 8\n"
            "x = lambda c: torch.rand((B, c, H, W), device=d)\n"
            "oa = x(3 * K)\n"
            "p = PropagationPlan(x(1), x(1), x(1), oa[:, 2 * K:], oa[:, :2 * K], torch.tensor([4.0], device=d))\n"
            "p.replay(); p.check(); p.close(); print('ok')\n") % os.path.dirname(os.path.dirname(__file__))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-3000:]
