"""Torch operator layer (layer 2): ``torch.ops.nlspn.*``.

The reference exposes its CUDA code through a pybind module (``DCN``,
src/model/deformconv/src/vision.cpp:6-13).  Here the same path is registered as
torch operators by ``csrc/nlspn_torch.cpp`` (libnlspn_torch.so, a thin C++ shim over
the C ABI in include/nlspn_prop.h), so calls go through the dispatcher instead of
ctypes, and TorchScript / ``torch.compile`` can see them.  The fake (meta) kernels
registered below give ``torch.compile`` the output shapes without running anything.

  torch.ops.nlspn.affinity_normalization(aff, gamma, kind)        nlspnmodel.py:179-201, :261-269
  torch.ops.nlspn.prop_step(feat, confidence, dep, aff, offset, kh, kw, raw_offsets,
                            preserve_input, always_clip)            :350-361 around :203-226
  torch.ops.nlspn.propagate(pred_init, dep, confidence, aff, offset, gamma, prop_time,
                            kh, kw, affinity, preserve_input, always_clip)
        -> (pred, pred_inter (T,B,1,H,W), aff, offset or None, confidence or None)   :323-381
  torch.ops.nlspn.modulated_deform_conv_forward / _backward        vision.cpp:9-10

The ops are inference building blocks (no autograd formula registered); the
differentiable forms stay ``nlspn_eccv20_amd.propagate`` / ``prop_step`` /
``dcn.ModulatedDeformConvFunction``.
"""
from __future__ import annotations

import os

import torch

from . import _lib

__all__ = ["load", "available"]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libnlspn_torch.so")
_loaded = False


def load() -> None:
    """Register torch.ops.nlspn.* (idempotent).  Raises if the library is missing:
    there is no fallback path."""
    global _loaded
    if _loaded:
        return
    _lib.get()  # libnlspn_hip.so first: the op library links against it
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    torch.ops.load_library(LIB_PATH)
    _register_fakes()
    _loaded = True


def available() -> bool:
    try:
        load()
        return True
    except (ImportError, OSError):
        return False


def _register_fakes() -> None:
    def fake_affnorm(aff, gamma, kind="TGASS"):
        B, K, H, W = aff.shape
        return aff.new_empty((B, K + 1, H, W))

    def fake_prop_step(feat, confidence, dep, aff, offset, kh=3, kw=3, raw_offsets=False, preserve_input=True,
                       always_clip=False):
        return torch.empty_like(feat)

    def fake_propagate(pred_init, dep, confidence, aff, offset, gamma, prop_time=18, kh=3, kw=3, affinity="TGASS",
                       preserve_input=True, always_clip=False):
        B, _, H, W = pred_init.shape
        K = kh * kw - 1
        e = pred_init.new_empty
        return (e((B, 1, H, W)), e((prop_time, B, 1, H, W)), e((B, K + 1, H, W)),
                e((B, 2 * (K + 1), H, W)) if offset is not None else None,
                e((B, 1, H, W)) if confidence is not None else None)

    def fake_mdcn_fwd(input, weight, bias, offset, mask, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                      dilation_h, dilation_w, group, deformable_group, im2col_step):
        B, _, H, W = input.shape
        Ho = (H + 2 * pad_h - (dilation_h * (kernel_h - 1) + 1)) // stride_h + 1
        Wo = (W + 2 * pad_w - (dilation_w * (kernel_w - 1) + 1)) // stride_w + 1
        return input.new_empty((B, weight.shape[0], Ho, Wo))

    def fake_mdcn_bwd(input, weight, bias, offset, mask, grad_output, *args):
        return [torch.empty_like(input), torch.empty_like(offset), torch.empty_like(mask), torch.empty_like(weight),
                torch.empty_like(bias)]

    for name, fn in (("affinity_normalization", fake_affnorm), ("prop_step", fake_prop_step),
                     ("propagate", fake_propagate), ("modulated_deform_conv_forward", fake_mdcn_fwd),
                     ("modulated_deform_conv_backward", fake_mdcn_bwd)):
        torch.library.register_fake(f"nlspn::{name}")(fn)
