"""S2D sparse-depth encoder front on the HIP kernel.

Reference: src/model/nlspnmodel.py:406-462 (class S2D).  ``s2d_front`` replaces the
pool pyramid (min pools 3/5/7/9 over the non-zero depths, :441-447; max pools 11/13,
:449-452), ``pool_convs`` (two 1x1 conv + ReLU, :455) and the
``torch.cat([dep_feat, dep], 1)`` (:459) with one fused kernel
(``nlspn_s2d_pyramid``, ``csrc/nlspn_s2d.h``); ``S2D.conv`` (the 3x3 conv) stays a
MIOpen convolution.  Differentiable in the four ``pool_convs`` parameters: the
kernel also writes the 6-channel pyramid, and the backward recomputes the two 1x1
layers from it in torch.  The sparse depth is data (no gradient), as in training.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from . import _lib

__all__ = ["s2d_front"]


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _run(dep, w1, b1, w2, b2, want_pyr):
    B, C, H, W = dep.shape
    if C != 1:
        raise RuntimeError(f"S2D expects a 1-channel sparse depth, got {tuple(dep.shape)}")
    for n, t in (("dep", dep), ("w1", w1), ("b1", b1), ("w2", w2), ("b2", b2)):
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a float32 CUDA tensor")
    if (tuple(w1.shape) != (8, 6, 1, 1) or tuple(w2.shape) != (16, 8, 1, 1) or b1.numel() != 8
            or b2.numel() != 16):
        raise RuntimeError("pool_convs must be Conv2d(6, 8, 1) and Conv2d(8, 16, 1) (nlspnmodel.py:423-426)")
    dep, w1, b1, w2, b2 = (t.contiguous() for t in (dep, w1, b1, w2, b2))
    out = torch.empty((B, 17, H, W), dtype=torch.float32, device=dep.device)
    pyr = torch.empty((B, 6, H, W), dtype=torch.float32, device=dep.device) if want_pyr else None
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    with torch.cuda.device(dep.device):
        _lib.check(_lib.get().nlspn_s2d_pyramid(_lib.DTYPE_F32, p(dep), p(w1), p(b1), p(w2), p(b2), p(out), p(pyr),
                                                B, H, W, _stream(dep.device)))
    return out, pyr


class _S2DFrontFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dep, w1, b1, w2, b2):
        out, pyr = _run(dep, w1, b1, w2, b2, want_pyr=True)
        ctx.save_for_backward(pyr, w1, b1, w2, b2)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_out):
        pyr, w1, b1, w2, b2 = ctx.saved_tensors
        with torch.enable_grad():
            params = [t.detach().requires_grad_(True) for t in (w1, b1, w2, b2)]
            h1 = F.relu(F.conv2d(pyr, params[0], params[1]))
            h2 = F.relu(F.conv2d(h1, params[2], params[3]))
            grads = torch.autograd.grad(h2, params, g_out[:, :16], allow_unused=True)
        return (None,) + tuple(grads)


def s2d_front(dep, w1, b1, w2, b2):
    """Pool pyramid + pool_convs + concat of S2D.forward (nlspnmodel.py:437-459):
    (B, 1, H, W) sparse depth -> (B, 17, H, W), the input of S2D.conv."""
    if torch.is_grad_enabled() and any(t.requires_grad for t in (w1, b1, w2, b2)):
        return _S2DFrontFn.apply(dep, w1, b1, w2, b2)
    return _run(dep, w1, b1, w2, b2, want_pyr=False)[0]
