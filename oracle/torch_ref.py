"""ORACLE (test infrastructure only) — the reference's own torch op sequence for the
NO-OFFSET propagation section, restated op for op for the CPU baseline.

Only ``tests/`` and ``bench.py``'s cpu_baseline leg may import this module.  It is
the timed CPU path SURVEY §8(d)(i) asks for: the reference's no-offset branch runs
on CPU as plain torch ops, so timing this sequence on the GPU box's host is timing
the reference's CPU path (the reference itself never travels to the box).

Op order follows src/model/nlspnmodel.py:
  _affinity_normalization  :179-201  (tanh / gamma, |.| sum + 1e-4, s<1 -> 1, divide)
  _aff_insert              :261-269  (ref tap = 1 - sum, inserted at K//2)
  forward prologue         :327-348  (mask_fix, confidence blend, first preserve/clip)
  loop body                :350-363  (feat * conf, _propagate_once, preserve, clip)
  _propagate_once no-offset:209-224  (replicate pad, 9 slices, cat, mul, sum)
  epilogue                 :375-377  (clamp(min=0) when not always_clip)
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def affinity_normalization(aff: torch.Tensor, gamma: float, kind: str = "TGASS") -> torch.Tensor:
    """:179-201 then :261-269."""
    if kind == "TC":
        aff = torch.tanh(aff) / gamma
    elif kind == "TGASS":
        aff = torch.tanh(aff) / (gamma + 1e-8)
    elif kind not in ("AS", "ASS"):
        raise NotImplementedError(kind)
    s = torch.sum(torch.abs(aff), dim=1, keepdim=True) + 1e-4
    if kind in ("ASS", "TGASS"):
        s[s < 1.0] = 1.0
    if kind != "TC":
        aff = aff / s
    K = aff.shape[1]
    ref = 1.0 - torch.sum(aff, dim=1, keepdim=True)
    taps = list(torch.chunk(aff, K, dim=1))
    taps.insert(K // 2, ref)
    return torch.cat(taps, dim=1)


def propagate_once_noffset(feat: torch.Tensor, aff: torch.Tensor) -> torch.Tensor:
    """:209-224 — 3x3 replicate-padded gather as nine shifted slices."""
    f = F.pad(feat, (1, 1, 1, 1), mode="replicate")
    H, W = f.shape[2], f.shape[3]
    sl = [f[:, :, dy:H - 2 + dy, dx:W - 2 + dx] for dy in range(3) for dx in range(3)]
    return torch.sum(torch.cat(sl, dim=1) * aff, dim=1, keepdim=True)


def propagate_noffset(pred_init, dep, conf, aff_raw, gamma, *, kind="TGASS", prop_time=18,
                      preserve_input=True, always_clip=False):
    """The whole no-offset section (:323-381) on CPU tensors; returns pred."""
    aff = affinity_normalization(aff_raw, gamma, kind)
    if preserve_input:
        m = (torch.sum(dep > 0.0, dim=1, keepdim=True) > 0.0).type_as(dep)
        if conf is not None:
            conf = (1.0 - m) * conf + m
    p = pred_init
    for k in range(1, prop_time + 1):
        if k == 1:
            if preserve_input:
                p = (1.0 - m) * p + m * dep
            if always_clip:
                p = torch.clamp(p, min=0)
        p = propagate_once_noffset(p * conf if conf is not None else p, aff)
        if preserve_input:
            p = (1.0 - m) * p + m * dep
        if always_clip:
            p = torch.clamp(p, min=0)
    return p if always_clip else torch.clamp(p, min=0)
