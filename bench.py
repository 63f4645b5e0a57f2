#!/usr/bin/env python3
"""Benchmark: NLSPN propagation iterations/s on MI355X (BASELINE.json metric).

One "step" = the whole propagation section of NLSPNModel.forward
(src/model/nlspnmodel.py:323-381) over one synthetic batch: the prologue
(affinity normalisation, offset insertion, confidence/input blend) plus T fused
iterations, replayed through a native plan (nlspn_plan_launch: step 1 + the
resident kernel re-issued directly, or the T step launches).  Inputs are
resident in HBM before the timed region.  value = iterations/s summed over all
ranks = N * T * steps / max-over-ranks wall time.

Workloads (BASELINE.json configs):
  headline (--config, default nyu) = C2: NYUv2 228x304, K=8, T=18, B=8, fp32,
      learned offsets (DCN path), TGASS — the configuration `value` is quoted on;
  "configs" object (same timing, roofline and PMC fields, per rank):
      C3 kitti    KITTI-DC 240x1216, K=8, T=18, B=4 fp32 (at N=8: C4, B=32 global),
      C5 nyu_k16  NYUv2, K=16 (1x17), T=36, B=16, fp16 storage,
      C1 nyu_b1   NYUv2 B=1 (the CPU config's workload, on the GPU).

Multi-GPU: `--gpus N` without a torchrun environment spawns N ranks itself
(nlspn_eccv20_amd.launch.spawn_local; the parent never touches the GPU).  Each rank
runs its own batch shard (weak scaling, no collective on the data path; SURVEY
§8e); the process group only carries the max-over-ranks timing and the per-rank
spread.  `--dry-run` runs the launcher and sharding logic on CPU (gloo, no GPU).

roofline (the dominant kernel: the resident kernel — iterations 2..T, one launch per
image group (C2: one group of 8 images; C3: two of 2) — where it applies, else the
per-iteration step kernel):
  achieved = COMPULSORY bytes per launch / its mean duration from dispatch-recorded
      HIP events (nlspn_time_propagate) on this stream.  Compulsory bytes are what
      the launch must move at least once: a step launch reads its 3K+3 input
      planes and writes one (SURVEY §8(d)'s S*(4+3K) per pixel); the resident launches
      read the 3K+2 invariant planes and p_1 once and write T-1 planes + pred (their
      duration spans every group's launch).
      So frac <= 1 for any kernel that really moves its bytes.
  alg_8d   = the secondary figure on SURVEY §8(d)'s per-iteration basis
      (S*(4+3K) bytes per pixel-iteration x the pixel-iterations of one launch),
      which credits the resident kernel with re-reads it does not do (can exceed 1).
  section  = the whole section's compulsory bytes (3K+3 planes read, T+3K+5
      written) / ms_per_step.
  traffic  = HBM-side bytes per launch from profiles/pmc_<config>.json (rocprofv3
      FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes), or null.
Extra objects (headline config only, not part of `value`): backward (fp32
forward+backward through autograd), gru_section (the reference's default GRU mode),
head_epilogue (the decoder's last three convs fused into one HIP kernel vs torch.cat + MIOpen),
cpu_baseline (rank 0, N=1; the C oracle for the offset path and the reference's
own torch op sequence for the no-offset path, all threads and 1 thread).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from nlspn_eccv20_amd import launch  # noqa: E402
from nlspn_eccv20_amd.sharding import gather_over_ranks, max_over_ranks, shard_range  # noqa: E402
from nlspn_eccv20_amd.synthetic import synth  # noqa: E402

CONFIGS = {
    "nyu": dict(id="C2", desc="NYUv2 228x304, K=8, T=18, B=8, fp32, learned offsets, TGASS",
                B=8, H=228, W=304, kernel=(3, 3), T=18, dtype="f32", max_depth=10.0, density=500 / (228 * 304)),
    "kitti": dict(id="C3", desc="KITTI-DC 240x1216, K=8, T=18, B=4, fp32, learned offsets, TGASS",
                  B=4, H=240, W=1216, kernel=(3, 3), T=18, dtype="f32", max_depth=90.0, density=0.05),
    "nyu_k16": dict(id="C5", desc="NYUv2 228x304, K=16 (1x17), T=36, B=16, fp16 storage, learned offsets, TGASS",
                    B=16, H=228, W=304, kernel=(1, 17), T=36, dtype="f16", max_depth=10.0, density=500 / (228 * 304)),
    "nyu_b1": dict(id="C1", desc="NYUv2 228x304, K=8, T=18, B=1, fp32, learned offsets, TGASS (C1's workload on "
                                 "the GPU)",
                   B=1, H=228, W=304, kernel=(3, 3), T=18, dtype="f32", max_depth=10.0, density=500 / (228 * 304)),
}
EXTRA = ("kitti", "nyu_k16", "nyu_b1")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
RESIDENT_FIRST = 0x100  # nlspn_time_propagate *resident bit: iteration 1 inside the resident launches


def baseline_metric():
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, KeyError, ValueError):
        return "propagation iters/sec (+ ms/iter)"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="nyu", choices=sorted(CONFIGS))
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-backward", action="store_true")
    ap.add_argument("--no-heads", action="store_true", help="skip the head-epilogue (fused conv) leg")
    ap.add_argument("--no-gru", action="store_true")
    ap.add_argument("--no-extra-configs", action="store_true")
    ap.add_argument("--backward-steps", type=int, default=20)
    ap.add_argument("--dry-run", action="store_true", help="launcher + sharding only, on CPU (gloo)")
    return ap.parse_args(argv)


def make_inputs(cfg, rank, dev):
    """Seeded synthetic head outputs of this rank's shard, in HBM."""
    tdt = torch.float16 if cfg["dtype"] == "f16" else torch.float32
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    s = synth(cfg["B"], cfg["H"], cfg["W"], K, seed=7240 + rank, density=cfg["density"], max_depth=cfg["max_depth"])
    to = lambda x: torch.from_numpy(x).to(dev, tdt)  # noqa: E731
    off_aff = to(s["off_aff"])
    inputs = {"pred_init": to(s["pred_init"]), "dep": to(s["dep"]), "conf": to(s["conf"]),
              "aff": off_aff[:, 2 * K:], "off": off_aff[:, :2 * K], "gamma": torch.tensor([0.5 * K], device=dev)}
    return inputs, s


def kernel_time(plan, inputs, cfg, reps, dev):
    """Dispatch-recorded HIP-event durations (nlspn_time_propagate) on this stream, over
    `reps` whole propagations on the plan's buffers: step 1 (prologue fused) and
    iterations 2..T — the resident-kernel launches (one per image group), or the sum of the T-1 step kernels."""
    from nlspn_eccv20_amd import _lib
    from nlspn_eccv20_amd.propagation import _ptr, _stream
    o = plan.outputs
    aff, off = inputs["aff"], inputs["off"]
    first, rest, res = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
    dt = _lib.DTYPE_F16 if cfg["dtype"] == "f16" else _lib.DTYPE_F32
    _lib.check(_lib.get().nlspn_time_propagate(
        dt, _ptr(inputs["pred_init"]), _ptr(inputs["dep"]), _ptr(inputs["conf"]), _ptr(aff), aff.stride(0),
        _ptr(off), off.stride(0), _ptr(inputs["gamma"]), _ptr(o["pred_inter"]), _ptr(o["pred"]), _ptr(o["aff"]),
        _ptr(o["offset"]), _ptr(o["confidence"]), _ptr(o["workspace"]), cfg["B"], cfg["H"], cfg["W"],
        cfg["kernel"][0], cfg["kernel"][1], cfg["T"], _lib.AFF_KINDS["TGASS"], _lib.PRESERVE_INPUT, reps,
        _stream(dev), ctypes.byref(first), ctypes.byref(rest), ctypes.byref(res)))
    return first.value, rest.value, int(res.value)


def pmc_traffic(config, kernel):
    """HBM-side bytes per launch of `kernel` from profiles/pmc_<config>.json (rocprofv3
    FETCH_SIZE/WRITE_SIZE passes, gfx950-corrected), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    entries = d.get("kernels", {d.get("kernel", ""): d})
    # the matching kernel launched most often: the per-iteration step kernel rather than
    # step 1 (which shares its name), the resident launches of every image group
    def first_step(name):  # prop_step_kernel<..., FIRST=true>: step 1, not the per-iteration kernel
        return name.split(">")[0].replace(" ", "").endswith(",true") and "prop_step_kernel" in name

    hits = [e for name, e in entries.items()
            if kernel in name and e.get("hbm_bytes_per_launch") and not first_step(name)]
    if not hits:
        return None
    return max(hits, key=lambda e: e.get("launches", 0)).get("hbm_bytes_per_launch")


def roofline(name, cfg, resident, first_ms, rest_ms, ms_per_step):
    """Roofline of the dominant kernel on compulsory bytes (frac <= 1), with the §8(d)
    per-iteration figure and the whole section beside it (see the module docstring)."""
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    T = cfg["T"]
    npx = cfg["B"] * cfg["H"] * cfg["W"]
    es = 2 if cfg["dtype"] == "f16" else 4
    plane = es * npx
    first_in = bool(resident & RESIDENT_FIRST)
    resident &= ~RESIDENT_FIRST
    if resident and first_in:
        kname, kmean = "prop_resident_kernel", rest_ms
        # the whole section: reads the raw head outputs (pred_init, conf, dep, K affinities,
        # 2K offsets); writes aff (K+1), offsets (2(K+1)), conf', pred_inter[0..T-1], pred
        comp_planes = (3 * K + 3) + (3 * K + 5 + T)
        alg_iters = T
        kdesc = (f"{kname} (prologue + iterations 1..{T}, invariant planes on chip: {resident} launch(es), the "
                 f"full image groups in turn inside one; kernel_ms_mean spans them all)")
    elif resident:
        kname, kmean = "prop_resident_kernel", rest_ms
        # reads: K normalised affinities (tap K/2 is recomputed), 2K offsets, conf', dep, p_1;
        # writes: pred_inter[1..T-1], pred and the output dict's 2(K+1) inserted-offset planes
        # (the resident loop copies them, one plane per iteration: ResArgs::off_out)
        comp_planes = (K + 2 * K + 2 + 1) + (T - 1 + 1) + 2 * (K + 1)
        alg_iters = T - 1
        kdesc = (f"{kname} (iterations 2..{T}, invariant planes on chip: {resident} launch(es), the full "
                 f"image groups in turn inside one; kernel_ms_mean spans them all)")
    else:
        kname, kmean = "prop_step_kernel", rest_ms / max(1, T - 1)
        comp_planes = 4 + 3 * K  # p_in, conf', dep, K aff, 2K offsets read; p_out written
        alg_iters = 1
        kdesc = f"{kname} (one fused iteration)"
    comp = comp_planes * plane
    achieved = comp / (kmean * 1e-3) / 1e9
    alg = es * (4 + 3 * K) * npx * alg_iters
    sec = ((3 * K + 3) + (T + 3 * K + 5)) * plane
    traffic = pmc_traffic(name, kname)
    if traffic and resident:
        traffic *= resident  # per launch -> the section's iterations 2..T (all launches)
    return {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kdesc,
        "bytes_basis": ("compulsory bytes of the prologue and iterations 1..T over all resident launches (each "
                        "plane read or written once)" if resident and first_in else
                        "compulsory bytes of iterations 2..T over all resident launches (each plane read or "
                        "written once)" if resident else
                        "compulsory bytes per launch (each plane the launch must read or write, once)"),
        "compulsory_bytes_per_launch": comp, "kernel_ms_mean": round(kmean, 5),
        # (no step-1 launch when the resident launches run the prologue: the interval is empty)
        "step1_kernel_ms": None if resident and first_in else round(first_ms, 5),
        "traffic_over_compulsory": round(traffic / comp, 3) if traffic else None,
        "alg_8d": {"bytes_per_launch": alg, "pixel_iterations_per_launch": npx * alg_iters,
                   "achieved": round(alg / (kmean * 1e-3) / 1e9, 1),
                   "frac": round(alg / (kmean * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "note": "SURVEY 8(d) S*(4+3K) per pixel-iteration; credits the resident kernel with the "
                           "invariant re-reads a per-iteration launch does, so it can exceed 1"},
        "section": {"compulsory_bytes": sec, "achieved": round(sec / (ms_per_step * 1e-3) / 1e9, 1),
                    "frac": round(sec / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "note": "whole section: raw head outputs read once, T pred_inter + pred + aff + offset + "
                            "confidence written once, over ms_per_step"},
    }


def measure(name, steps, warmup, kernel_reps, world, rank, dev):
    """Time one workload on every rank (barrier + synchronize on both sides, max over
    ranks) and its dominant kernel; returns (result dict, inputs, synthetic arrays)."""
    from nlspn_eccv20_amd.propagation import PropagationPlan
    cfg = CONFIGS[name]
    inputs, s = make_inputs(cfg, rank, dev)
    plan = PropagationPlan(inputs["pred_init"], inputs["dep"], inputs["conf"], inputs["aff"], inputs["off"],
                           inputs["gamma"], prop_time=cfg["T"], kernel=cfg["kernel"])
    for _ in range(warmup):
        plan.replay()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        plan.replay()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    mine = time.perf_counter() - t0
    plan.check()  # a resident launch that aborted raises here (never silent)
    spread = gather_over_ranks(mine, dev)
    elapsed = max_over_ranks(mine, dev)
    first_ms, rest_ms, resident = kernel_time(plan, inputs, cfg, kernel_reps, dev)
    plan.check()
    plan.close()
    ms_per_step = 1e3 * elapsed / steps
    out = {
        "workload": f"{cfg['id']}: {cfg['desc']}",
        "value": round(world * cfg["T"] * steps / elapsed, 1), "unit": "iters/s",
        "ms_per_step": round(ms_per_step, 4), "ms_per_iter": round(ms_per_step / cfg["T"], 5),
        "dtype": cfg["dtype"], "batch_per_gpu": cfg["B"], "global_batch": cfg["B"] * world,
        "shard": list(shard_range(cfg["B"] * world, world, rank)),
        "gpu_event_ms_per_step": round(ev0.elapsed_time(ev1) / steps, 4),
        "rank_ms_per_step": [round(1e3 * x / steps, 4) for x in spread],
        "roofline": roofline(name, cfg, resident, first_ms, rest_ms, ms_per_step),
    }
    return out, inputs, s


def backward_timing(inputs, cfg, steps):
    """Forward+backward of the whole section (training step of the propagation), with
    gradients for pred_init, confidence, the (B, 3K, H, W) head output and gamma."""
    from nlspn_eccv20_amd.propagation import propagate
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    pi = inputs["pred_init"].detach().clone().requires_grad_(True)
    cf = inputs["conf"].detach().clone().requires_grad_(True)
    oa = torch.cat([inputs["off"], inputs["aff"]], 1).detach().requires_grad_(True)
    g = inputs["gamma"].detach().clone().requires_grad_(True)
    gp = torch.randn_like(pi)

    def fwd():
        return propagate(pi, inputs["dep"], cf, oa[:, 2 * K:], oa[:, :2 * K], g, prop_time=cfg["T"],
                         kernel=cfg["kernel"])

    def train_step():
        torch.autograd.backward(fwd()["pred"], gp)

    for _ in range(3):
        train_step()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    torch.cuda.synchronize()
    e[0].record()
    for _ in range(steps):
        train_step()
    e[1].record()
    with torch.no_grad():
        e[2].record()
        for _ in range(steps):
            fwd()
        e[3].record()
    torch.cuda.synchronize()
    fb = e[0].elapsed_time(e[1]) / steps
    fo = e[2].elapsed_time(e[3]) / steps
    out = {"ms_fwd_bwd_per_step": round(fb, 4), "ms_fwd_per_step": round(fo, 4),
           "ms_bwd_per_iter": round((fb - fo) / cfg["T"], 5), "steps": steps,
           "note": "eager autograd; bwd = fwd+bwd - fwd. graph: the same training step and forward captured "
                   "into hipGraphs (torch.cuda.graph, whole step incl. autograd backward) and replayed"}
    try:  # graph-replayed: no host launch gaps between the backward's per-iteration kernels
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                for t in (pi, cf, oa, g):
                    t.grad = None
                train_step()
        torch.cuda.current_stream().wait_stream(side)
        for t in (pi, cf, oa, g):
            t.grad = None
        gtrain, gfwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gtrain):
            train_step()
        with torch.no_grad(), torch.cuda.graph(gfwd):
            fwd()
        for gr in (gtrain, gfwd):
            gr.replay()
        torch.cuda.synchronize()
        e[0].record()
        for _ in range(steps):
            gtrain.replay()
        e[1].record()
        e[2].record()
        for _ in range(steps):
            gfwd.replay()
        e[3].record()
        torch.cuda.synchronize()
        fbg = e[0].elapsed_time(e[1]) / steps
        fog = e[2].elapsed_time(e[3]) / steps
        out.update({"ms_fwd_bwd_per_step_graph": round(fbg, 4), "ms_fwd_per_step_graph": round(fog, 4),
                    "ms_bwd_per_iter_graph": round((fbg - fog) / cfg["T"], 5)})
    except Exception as ex:  # noqa: BLE001  (report, do not fail the bench line)
        out["graph_error"] = f"{type(ex).__name__}: {ex}"[:300]
    return out


def gru_section_timing(inputs, cfg, steps, dev):
    """GRU mode (the reference's forced default, src/config.py:225-228): the section of
    NLSPNModel (nlspnmodel.py:303-383, ConvGRU re-estimating the affinity every
    iteration) on the bench's synthetic head outputs, random-init GRU weights, eager
    vs captured into one hipGraph (SectionGraph).  Not part of `value`."""
    import types
    from nlspn_eccv20_amd import NLSPNModel, SectionGraph
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    args = types.SimpleNamespace(prop_kernel=cfg["kernel"][0], affinity="TGASS", affinity_gamma=0.5,
                                 prop_time=cfg["T"], preserve_input=True, always_clip=False, conf_prop=True,
                                 offset=True, network="resnet34", from_scratch=True, zero_init_aff=False,
                                 use_GRU=True, use_S2D=False, GRU_hidden_dim=128, GRU_input_dim=128, lr=1e-3,
                                 max_depth=cfg["max_depth"], patch_height=cfg["H"], patch_width=cfg["W"],
                                 model_name="NLSPN")
    torch.manual_seed(0)
    m = NLSPNModel(args).to(dev).eval()
    off_aff = torch.cat([inputs["off"], inputs["aff"]], 1).contiguous()
    heads = (inputs["pred_init"], off_aff, inputs["conf"], inputs["dep"])
    assert off_aff.shape[1] == 3 * K
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def timed(native):
        m.native_gru = native
        g = SectionGraph(m, *heads)
        with torch.no_grad():
            for _ in range(3):
                m.propagate_heads(*heads)
                g.replay()
            torch.cuda.synchronize()
            e[0].record()
            for _ in range(steps):
                m.propagate_heads(*heads)
            e[1].record()
            e[2].record()
            for _ in range(steps):
                g.replay()
            e[3].record()
        torch.cuda.synchronize()
        del g
        return e[0].elapsed_time(e[1]) / steps, e[2].elapsed_time(e[3]) / steps

    # the GRU-mode convolutions on the HIP kernels (gru.py, the model's inference default) ...
    eager, graph = timed(True)
    # ... and on the torch modules (MIOpen), NCHW with MIOpen's default algorithms
    m_eager, m_graph = timed(False)
    # the modules with the GRU convolutions in channels_last and MIOpen's algorithm search on
    # (NLSPNModel.gru_channels_last; cudnn.benchmark restored afterwards)
    prev = torch.backends.cudnn.benchmark
    torch.backends.cudnn.benchmark = True
    try:
        m.native_gru = False
        m.gru_channels_last()
        g = SectionGraph(m, *heads)
        with torch.no_grad():
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e[0].record()
            for _ in range(steps):
                g.replay()
            e[1].record()
        torch.cuda.synchronize()
        tuned = e[0].elapsed_time(e[1]) / steps
    finally:
        torch.backends.cudnn.benchmark = prev
    return {"ms_per_step_eager": round(eager, 4), "ms_per_step_graph": round(graph, 4),
            "iters_per_s_graph": round(cfg["T"] / (graph * 1e-3), 1),
            "modules": {"ms_per_step_eager": round(m_eager, 4), "ms_per_step_graph": round(m_graph, 4),
                        "ms_per_step_graph_channels_last_tuned": round(tuned, 4)},
            "speedup_vs_tuned_modules": round(tuned / graph, 3), "steps": steps,
            "note": "per iteration: encode_dep, ConvGRU (hidden 128), decode_aff + crop as HIP f32-MFMA convolutions "
                    "(gru.py; the first update also encode_aff), the affinity normalisation in the last conv's epilogue (K = 8), prop_step; graph = one "
                    "hipGraph replay of the section (SectionGraph). modules: the same section on the torch modules "
                    "(MIOpen), default and channels_last + MIOpen algorithm search"}


def head_epilogue_timing(cfg, dev, reps=20):
    """The head epilogue (nlspnmodel.py:296-315): the decoder's last
    three 3x3 convs (off_aff_dec0 -> 3K, id_dec0 -> 1 + ReLU, cf_dec0 -> 1 + Sigmoid) on
    fe1 and the three 64-channel decoder outputs, at this config's B x H x W, fused HIP
    kernel (nlspn_head_epilogue) vs the reference's op sequence on torch (torch.cat +
    MIOpen conv + activation).  Synthetic U(0,1) activations, default-init weights; CUDA
    events, median of `reps` after 5 warm-ups.  Not part of `value`."""
    import torch.nn as nn
    from nlspn_eccv20_amd.heads import HeadWeights, head_epilogue
    B, H, W = cfg["B"], cfg["H"], cfg["W"]
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    g = torch.Generator(device=dev).manual_seed(11)
    fe1, id_fd1, oa_fd1, cf_fd1 = (torch.rand((B, 64, H, W), device=dev, generator=g) for _ in range(4))
    torch.manual_seed(11)
    oa, idc, cfc = (nn.Conv2d(128, n, 3, padding=1).to(dev) for n in (3 * K, 1, 1))
    hw = HeadWeights()

    def fused():
        return head_epilogue(fe1, oa_fd1, oa, id_fd1, idc, cf_fd1, cfc, weights=hw)

    def ref():
        return (torch.relu(idc(torch.cat((id_fd1, fe1), 1))), oa(torch.cat((oa_fd1, fe1), 1)),
                torch.sigmoid(cfc(torch.cat((cf_fd1, fe1), 1))))

    def med(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    # heads + propagation section: raw epilogue then nlspn_propagate (step 1 normalises)
    # vs the epilogue with the prologue fused in then nlspn_propagate_normalized
    from nlspn_eccv20_amd import propagate, propagate_normalized
    from nlspn_eccv20_amd.heads import head_epilogue_prologue
    dep = torch.rand((B, 1, H, W), device=dev, generator=g) * cfg["max_depth"]
    dep = dep * (torch.rand((B, 1, H, W), device=dev, generator=g) < cfg["density"])
    gamma = torch.tensor([0.5 * K], device=dev)
    kern = cfg["kernel"]

    def unfused_section():
        pi, oa_out, co = fused()
        return propagate(pi, dep, co, oa_out[:, 2 * K:], oa_out[:, :2 * K], gamma, prop_time=cfg["T"],
                         kernel=kern)["pred"]

    def fused_section():
        h = head_epilogue_prologue(fe1, oa_fd1, oa, id_fd1, idc, dep, gamma, "TGASS", cf_fd1, cfc, weights=hw)
        return propagate_normalized(h["p0"], dep, h["confidence"], h["aff"], h["offset"], cfg["T"], kern)["pred"]

    with torch.no_grad():
        t_fused, t_ref = med(fused), med(ref)
        f, r = fused(), ref()
        diff = max((a - b).abs().max().item() for a, b in zip(f, r))
        sec = {}
        if kern == (3, 3):
            sec = {"ms_heads_then_propagate": round(med(unfused_section), 4),
                   "ms_heads_prologue_then_loop": round(med(fused_section), 4),
                   "bit_identical_pred": bool(torch.equal(unfused_section(), fused_section()))}
    del fe1, id_fd1, oa_fd1, cf_fd1
    flops = 2.0 * B * H * W * 128 * 9 * (3 * K + 2)
    ach = flops / (t_fused * 1e-3) / 1e12
    return {"ms_fused": round(t_fused, 4), "ms_torch": round(t_ref, 4), "speedup": round(t_ref / t_fused, 2),
            "max_abs_diff_vs_torch": diff,
            "roofline": {"bound": "mfma", "achieved": round(ach, 2), "peak": 157.3, "unit": "TFLOP/s",
                         "frac": round(ach / 157.3, 3),
                         "basis": "useful FLOPs 2*B*H*W*128*9*(3K+2) / fused-call time; peak = f32-input MFMA "
                                  "(v_mfma_f32_32x32x2_f32, MI355X_MICROARCH.md)"},
            "with_section": sec,
            "note": "fused: one HIP kernel (nlspn_heads.h, f32 operands on the matrix cores), reads fe1 + decoder "
                    "outputs in place; torch: 3 x (torch.cat + MIOpen conv) + ReLU/Sigmoid; with_section: the heads "
                    "then the T-iteration section, eager, raw epilogue + nlspn_propagate vs the epilogue with the "
                    "prologue fused in + nlspn_propagate_normalized"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _median_time(fn, reps, warm):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def cpu_baseline(reps, warm=2):
    """SURVEY §8(d) CPU baseline on this host, rank 0, N=1: (i) the offset path through
    the C oracle (kind "port": the reference has no CPU DCN) and (ii) the no-offset path
    as the reference's own torch op sequence (nlspnmodel.py:209-224, oracle/torch_ref.py),
    each at the C2 batch and the C1 batch (B=1) with all threads of this process's CPU
    share, and at C1 with 1 thread; 2 warm-ups, median of `reps` whole sections."""
    from oracle import oracle as O  # test infrastructure: the CPU baseline leg only
    from oracle import torch_ref
    host = os.cpu_count() or 1
    # the GPU box gives one GPU's job a 16-core share (OMP_NUM_THREADS there); use it all
    threads = max(1, min(host, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    legs = {}
    for name in ("nyu", "nyu_b1"):
        cfg = CONFIGS[name]
        K = cfg["kernel"][0] * cfg["kernel"][1] - 1
        s = synth(cfg["B"], cfg["H"], cfg["W"], K, seed=7240, density=cfg["density"], max_depth=cfg["max_depth"])
        a_off = (s["pred_init"], s["dep"], s["conf"], s["off_aff"][:, 2 * K:], s["off_aff"][:, :2 * K], 0.5 * K)
        tt = {k: torch.from_numpy(s[k]) for k in ("pred_init", "dep", "conf")}
        aff_t = torch.from_numpy(s["off_aff"][:, 2 * K:].copy())
        for nth in ((threads, 1) if name == "nyu_b1" else (threads,)):
            O.set_threads(nth)
            torch.set_num_threads(nth)
            med = _median_time(lambda: O.propagate(*a_off, prop_time=cfg["T"]), reps, warm)
            legs[f"offset_{cfg['id']}_{nth}t"] = {"iters_per_s": round(cfg["T"] / med, 2),
                                                   "ms_per_iter": round(1e3 * med / cfg["T"], 3)}
            med = _median_time(lambda: torch_ref.propagate_noffset(tt["pred_init"], tt["dep"], tt["conf"], aff_t,
                                                                   0.5 * K, prop_time=cfg["T"]), reps, warm)
            legs[f"noffset_{cfg['id']}_{nth}t"] = {"iters_per_s": round(cfg["T"] / med, 2),
                                                    "ms_per_iter": round(1e3 * med / cfg["T"], 3)}
    head = legs[f"offset_C2_{threads}t"]
    return {"value": head["iters_per_s"], "unit": "iters/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(), "host_logical_cpus": host,
            "sample": (f"C2 workload (NYU B=8, K=8, T=18, fp32, learned offsets, TGASS) through the C oracle "
                       f"(oracle/nlspn_oracle.c, OpenMP {threads} threads = this job's CPU share), {warm} warm-ups + "
                       f"median of {reps} whole sections; legs: offset path (C oracle) and no-offset path (the "
                       f"reference's torch op sequence, nlspnmodel.py:209-224) at C2 and C1 (B=1) with {threads} "
                       f"threads and C1 with 1 thread"),
            "ms_per_iter": head["ms_per_iter"], "legs": legs}


def dry_run(a, world, rank):
    """Launcher + sharding on CPU (gloo): every rank owns its shard of the global batch
    and reports it; rank 0 prints one JSON line.  No GPU is touched."""
    launch.init_from_env("gloo")
    cfg = CONFIGS[a.config]
    lo, hi = shard_range(cfg["B"] * world, world, rank)
    t0 = time.perf_counter()
    K = cfg["kernel"][0] * cfg["kernel"][1] - 1
    s = synth(hi - lo, 8, 8, K, seed=7240 + rank)
    mine = time.perf_counter() - t0
    shards = [None] * world
    if world > 1:
        dist.all_gather_object(shards, (rank, lo, hi, float(s["pred_init"].sum())))
    else:
        shards = [(rank, lo, hi, float(s["pred_init"].sum()))]
    el = max_over_ranks(mine)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "config": cfg["id"], "global_batch": cfg["B"] * world,
                          "shards": [[r, l, h] for r, l, h, _ in shards], "max_rank_s": el}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, spawned here (the parent never initialises HIP)
        sys.exit(launch.spawn_local(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world, rank, local = launch.env_rank()
    if a.dry_run:
        return dry_run(a, world, rank)
    if a.gpus != world:
        print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}; reporting the {world} ranks that run",
              file=sys.stderr)
    launch.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cfg = CONFIGS[a.config]

    head, inputs, _ = measure(a.config, a.steps, a.warmup, a.kernel_reps, world, rank, dev)
    out = {
        "metric": baseline_metric(),
        "value": head["value"], "unit": "iters/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"], "ms_per_iter": head["ms_per_iter"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": cfg["dtype"],
        "data": "synthetic (seeded; SURVEY §8d distribution, convex |N(0,1)| affinity, N(0,2^2) offsets)",
        "config": {"workload": head["workload"], "batch_per_gpu": cfg["B"], "global_batch": cfg["B"] * world,
                   "H": cfg["H"], "W": cfg["W"], "K": cfg["kernel"][0] * cfg["kernel"][1] - 1,
                   "kernel": list(cfg["kernel"]), "prop_time": cfg["T"],
                   "parallelism": f"dp{world} (batch shards, no collective)"},
        "roofline": head["roofline"],
        "gpu_event_ms_per_step": head["gpu_event_ms_per_step"],
        "rank_ms_per_step": head["rank_ms_per_step"],
    }
    if cfg["dtype"] == "f32" and not a.no_backward:
        out["backward"] = backward_timing(inputs, cfg, a.backward_steps)
    if cfg["dtype"] == "f32" and cfg["kernel"] == (3, 3) and not a.no_gru:
        out["gru_section"] = gru_section_timing(inputs, cfg, a.backward_steps, dev)
    del inputs
    if cfg["dtype"] == "f32" and not a.no_heads:
        out["head_epilogue"] = head_epilogue_timing(cfg, dev)
        torch.cuda.empty_cache()
    if not a.no_extra_configs:
        out["configs"] = {}
        for name in EXTRA:
            if name == a.config:
                continue
            r, _, _ = measure(name, a.steps, a.warmup, a.kernel_reps, world, rank, dev)
            out["configs"][CONFIGS[name]["id"]] = r
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.cpu_reps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
