"""Real-data replay of the propagation section from the reference's summary dumps.

The reference's summary writer saves, for each logged sample, the learned planes the
propagation ran on (src/summary/nlspnsummary.py:185-189 takes them from the output
dict, :265-268 writes them):

  offset.npy  output['offset']: the inserted layout (B, 2(K+1), H, W) (_off_insert,
              nlspnmodel.py:252-259); absent when the model runs without offsets
  aff.npy     output['aff']: the normalised affinity (B, K+1, H, W), reference tap at
              K//2 (nlspnmodel.py:179-201, :261-269)
  gamma.npy   output['gamma']: aff_scale_const, shape (1,)

load_dump() reads them as data only (numpy, allow_pickle=False), save_dump() writes an
output dict of this package (or of the reference) in the same three files, and replay()
re-runs the T-iteration loop (nlspnmodel.py:327-381) on the HIP path from the dumped
planes plus the caller's pred_init / dep / confidence.  Recorded offsets and affinities
can so be timed and parity-checked instead of synthetic ones.

The dumped affinity is the one the LAST iteration used: in GRU mode (use_GRU,
nlspnmodel.py:365-373) it changes every iteration, so a replay of a GRU-mode dump is a
plain (fixed-affinity) section on that affinity, not the recorded run.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from . import propagation as P

__all__ = ["SummaryDump", "load_dump", "save_dump", "replay"]

@dataclass
class SummaryDump:
    """The planes of one summary dump (float32, as the reference saves them)."""
    aff: np.ndarray                 # (B, K+1, H, W), normalised
    offset: Optional[np.ndarray]    # (B, 2(K+1), H, W), inserted layout, or None
    gamma: np.ndarray               # (1,)
    kernel: Tuple[int, int]         # (kh, kw), kh * kw = K + 1

    @property
    def K(self) -> int:
        return self.aff.shape[1] - 1

    @property
    def shape(self) -> Tuple[int, int, int]:
        B, _, H, W = self.aff.shape
        return B, H, W


def _load(path: str) -> np.ndarray:
    a = np.load(path, allow_pickle=False)  # data only: a pickled object array is refused
    if a.dtype.kind != "f":
        raise ValueError(f"{path}: expected a floating-point array, got {a.dtype}")
    return np.ascontiguousarray(a, dtype=np.float32)


def _infer_kernel(taps: int, kernel) -> Tuple[int, int]:
    if kernel is not None:
        kh, kw = P.kernel_geometry(kernel)
        if kh * kw != taps:
            raise ValueError(f"kernel {kh}x{kw} has {kh * kw} taps, the dumped affinity has {taps}")
        return kh, kw
    k = int(round(math.sqrt(taps)))
    if k * k != taps or k % 2 == 0:
        raise ValueError(f"cannot infer a square odd kernel from {taps} taps; pass kernel=(kh, kw)")
    return k, k


def load_dump(path: str, kernel=None) -> SummaryDump:
    """Read offset.npy (optional), aff.npy and gamma.npy from a summary output directory
    (nlspnsummary.py:265-268).  kernel: (kh, kw) when K + 1 is not an odd square (the
    1x17 geometry of config C5); otherwise inferred as the reference does (prop_kernel k,
    K = k*k - 1, nlspnmodel.py:29-32)."""
    ap = os.path.join(path, "aff.npy")
    gp = os.path.join(path, "gamma.npy")
    op = os.path.join(path, "offset.npy")
    for p in (ap, gp):
        if not os.path.isfile(p):
            raise FileNotFoundError(f"summary dump is missing {p}")
    aff = _load(ap)
    if aff.ndim != 4 or aff.shape[1] < 2:
        raise ValueError(f"aff.npy must be (B, K+1, H, W), got {aff.shape}")
    B, taps, H, W = aff.shape
    kh, kw = _infer_kernel(taps, kernel)
    gamma = _load(gp).reshape(-1)
    if gamma.shape != (1,):
        raise ValueError(f"gamma.npy must hold one value, got shape {gamma.shape}")
    off = None
    if os.path.isfile(op):
        off = _load(op)
        if off.shape != (B, 2 * taps, H, W):
            raise ValueError(f"offset.npy must be {(B, 2 * taps, H, W)} (inserted layout), got {off.shape}")
        ref = taps // 2
        if np.any(off[:, 2 * ref:2 * ref + 2] != 0):
            raise ValueError("offset.npy: the reference tap's (dh, dw) planes are not zero; "
                             "expected the inserted layout of _off_insert")
    elif kh * kw != 9:
        raise ValueError("a dump without offset.npy takes the no-offset branch, which is 3x3 only "
                         "(nlspnmodel.py:209-224)")
    return SummaryDump(aff=aff, offset=off, gamma=gamma, kernel=(kh, kw))


def save_dump(path: str, output: dict) -> None:
    """Write output['offset'] / ['aff'] / ['gamma'] as the reference's summary does
    (nlspnsummary.py:185-189, :265-268): offset.npy only when the output has offsets."""
    os.makedirs(path, exist_ok=True)
    off = output.get("offset")
    if off is not None:
        np.save(os.path.join(path, "offset.npy"), off.detach().float().cpu().numpy())
    np.save(os.path.join(path, "aff.npy"), output["aff"].detach().float().cpu().numpy())
    np.save(os.path.join(path, "gamma.npy"), output["gamma"].detach().float().cpu().numpy().reshape(1))


def _dev(x, device, dtype):
    if x is None:
        return None
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))
    return t.to(device=device, dtype=dtype).contiguous()


def replay(dump: SummaryDump, pred_init, dep, confidence=None, *, prop_time: int = 18,
           preserve_input: bool = True, always_clip: bool = False, device="cuda",
           dtype: torch.dtype = torch.float32) -> dict:
    """Re-run the propagation section on a dump's affinity / offsets (inference).

    pred_init, dep, confidence: (B, 1, H, W) arrays or tensors of the dump's B, H, W;
    confidence is the raw head output (None: conf_prop off).  The prologue is the
    reference's (nlspnmodel.py:327-348): m = [dep > 0], conf' = (1-m) conf + m,
    p0 = (1-m) pred_init + m dep, clamped with always_clip; then T iterations on the
    HIP path — propagate_normalized with offsets, prop_step's no-offset branch without.
    dtype: plane storage (float32, or float16 with fp32 math).
    Returns the reference's output dict keys: pred, pred_init, pred_inter (T views),
    offset, aff, gamma, confidence (blended) — and pred_inter_tensor."""
    B, H, W = dump.shape
    kh, kw = dump.kernel
    T = int(prop_time)
    if T < 1:
        raise ValueError(f"prop_time must be >= 1, got {prop_time}")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("replay runs on the HIP path: device must be a CUDA (HIP) device")
    p = _dev(pred_init, dev, dtype)
    d = _dev(dep, dev, dtype)
    c = _dev(confidence, dev, dtype)
    for n, t in (("pred_init", p), ("dep", d), ("confidence", c)):
        if t is not None and tuple(t.shape) != (B, 1, H, W):
            raise ValueError(f"{n} must be {(B, 1, H, W)} to match the dump, got {tuple(t.shape)}")
    if preserve_input and d is None:
        raise RuntimeError("preserve_input requires dep")
    aff = _dev(dump.aff, dev, dtype)
    off = _dev(dump.offset, dev, dtype)

    p0 = p
    if preserve_input:  # :328-334, :343-345, in the reference's operation order
        m = (d > 0.0).to(dtype)
        if c is not None:
            c = (1.0 - m) * c + m
        p0 = (1.0 - m) * p0 + m * d
    if always_clip:
        p0 = torch.clamp(p0, min=0)

    if off is not None:
        o = P.propagate_normalized(p0.contiguous(), d, c, aff, off, prop_time=T, kernel=(kh, kw),
                                   preserve_input=preserve_input, always_clip=always_clip)
        pred_inter, pred = o["pred_inter_tensor"], o["pred"]
    else:
        pred_inter = torch.empty((T, B, 1, H, W), dtype=dtype, device=dev)
        pred = torch.empty((B, 1, H, W), dtype=dtype, device=dev)
        src = p0.contiguous()
        for t in range(T):
            P.prop_step(src, c, d, aff, None, preserve_input=preserve_input, always_clip=always_clip,
                        out=pred_inter[t], pred_out=pred if t == T - 1 else None)
            src = pred_inter[t]
    gamma = torch.from_numpy(dump.gamma.copy()).to(dev)
    return {"pred": pred, "pred_init": p, "pred_inter": list(pred_inter.unbind(0)), "offset": off, "aff": aff,
            "gamma": gamma, "confidence": c, "pred_inter_tensor": pred_inter}
