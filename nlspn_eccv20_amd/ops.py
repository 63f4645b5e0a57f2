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
  torch.ops.nlspn.propagate_normalized(p0, dep, confidence, aff, offset, prop_time, kh, kw,
                                       preserve_input, always_clip) -> (pred, pred_inter)
        the loop from prologued inputs (normalised (K+1)-tap affinity, inserted offsets:
        what the fused head epilogue writes), :340-381; inference only
  torch.ops.nlspn.modulated_deform_conv_forward / _backward        vision.cpp:9-10

Autograd (round 3): every forward op has a backward registered
(torch.library.register_autograd), built on the same HIP backward entry points as the
ctypes autograd functions of propagation.py / dcn.py — the reference's DCN is
differentiable wherever ModulatedDeformConvFunction appears
(modulated_deform_conv_func.py:38-56).  The backward passes are ops too, so
torch.compile traces a training step through them:

  torch.ops.nlspn.propagate_backward             nlspn_propagate_backward (the section)
  torch.ops.nlspn.prop_step_backward             nlspn_prop_step_backward (raw offsets, float32)
  torch.ops.nlspn.affinity_normalization_backward  nlspn_affinity_normalize_backward
  torch.ops.nlspn.modulated_deform_conv_backward  (the seam-2 op above)

Gradients flow from pred / pred_inter of ``propagate`` (its aff / offset / confidence
outputs are the output dict's copies and take no gradient, as in propagation.propagate).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch import Tensor

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
    _register_autograd()
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

    def fake_propagate_normalized(p0, dep, confidence, aff, offset, prop_time=18, kh=3, kw=3, preserve_input=True,
                                  always_clip=False):
        B, _, H, W = p0.shape
        return p0.new_empty((B, 1, H, W)), p0.new_empty((prop_time, B, 1, H, W))

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
                     ("propagate", fake_propagate), ("propagate_normalized", fake_propagate_normalized),
                     ("modulated_deform_conv_forward", fake_mdcn_fwd),
                     ("modulated_deform_conv_backward", fake_mdcn_bwd)):
        torch.library.register_fake(f"nlspn::{name}")(fn)


def _register_autograd() -> None:
    from . import propagation as P

    def _z(t):
        return t.new_empty((0,))

    # ---- backward ops (custom ops over the ctypes backward paths; fake kernels for compile)
    @torch.library.custom_op("nlspn::propagate_backward", mutates_args=())
    def propagate_backward(pred_init: Tensor, dep: Optional[Tensor], confidence: Optional[Tensor], aff: Tensor,
                           offset: Optional[Tensor], gamma: Tensor, pred_inter: Tensor, aff_norm: Tensor,
                           conf_eff: Optional[Tensor], g_pred: Optional[Tensor], g_inter: Optional[Tensor], kh: int,
                           kw: int, affinity: str, preserve_input: bool,
                           always_clip: bool) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
        g_pi, g_conf, g_aff, g_off, g_gamma, _ = P._section_backward(
            pred_init, dep, confidence, aff, offset, gamma, pred_inter, aff_norm, conf_eff, g_pred, g_inter, kh, kw,
            pred_inter.shape[0], affinity, preserve_input, always_clip)
        return (g_pi, _z(pred_init) if g_conf is None else g_conf, g_aff, _z(pred_init) if g_off is None else g_off,
                torch.zeros_like(gamma) if g_gamma is None else g_gamma)

    @propagate_backward.register_fake
    def _(pred_init, dep, confidence, aff, offset, gamma, pred_inter, aff_norm, conf_eff, g_pred, g_inter, kh, kw,
          affinity, preserve_input, always_clip):
        B, _, H, W = pred_init.shape
        K = kh * kw - 1
        e = pred_init.new_empty
        return (e((B, 1, H, W)), e((B, 1, H, W)) if confidence is not None else e((0,)), e((B, K, H, W)),
                e((B, 2 * K, H, W)) if offset is not None else e((0,)), torch.empty_like(gamma))

    @torch.library.custom_op("nlspn::prop_step_backward", mutates_args=())
    def prop_step_backward(feat: Tensor, confidence: Optional[Tensor], dep: Optional[Tensor], aff: Tensor,
                           offset: Optional[Tensor], g_out: Tensor, kh: int, kw: int, preserve_input: bool,
                           always_clip: bool) -> tuple[Tensor, Tensor, Tensor, Tensor]:
        g_feat, g_conf, g_aff, g_off = P._step_backward(feat, confidence, dep, aff, offset, g_out, kh, kw,
                                                        preserve_input, always_clip)
        return g_feat, _z(feat) if g_conf is None else g_conf, g_aff, _z(feat) if g_off is None else g_off

    @prop_step_backward.register_fake
    def _(feat, confidence, dep, aff, offset, g_out, kh, kw, preserve_input, always_clip):
        B, _, H, W = feat.shape
        K = kh * kw - 1
        e = feat.new_empty
        return (e((B, 1, H, W)), e((B, 1, H, W)) if confidence is not None else e((0,)), e((B, K + 1, H, W)),
                e((B, 2 * K, H, W)) if offset is not None else e((0,)))

    @torch.library.custom_op("nlspn::affinity_normalization_backward", mutates_args=())
    def affinity_normalization_backward(aff: Tensor, gamma: Tensor, g_out: Tensor,
                                        kind: str) -> tuple[Tensor, Tensor]:
        g_raw, g_gamma = P._affnorm_backward(aff, gamma, g_out, kind)
        return g_raw, torch.zeros_like(gamma) if g_gamma is None else g_gamma

    @affinity_normalization_backward.register_fake
    def _(aff, gamma, g_out, kind):
        return torch.empty_like(aff, dtype=torch.float32), torch.empty_like(gamma)

    # ---- autograd of the forward ops
    def setup_propagate(ctx, inputs, output):
        pred_init, dep, confidence, aff, offset, gamma, _T, kh, kw, affinity, preserve_input, always_clip = inputs
        _pred, pred_inter, aff_out, _off, conf_out = output
        ctx.save_for_backward(pred_init, dep, confidence, aff, offset, gamma, pred_inter, aff_out, conf_out)
        ctx.cfg = (kh, kw, affinity, preserve_input, always_clip)

    def bwd_propagate(ctx, g_pred, g_inter, _g_aff, _g_off, _g_conf):
        pred_init, dep, confidence, aff, offset, gamma, pred_inter, aff_out, conf_out = ctx.saved_tensors
        kh, kw, affinity, pre, clip = ctx.cfg
        gp, gc, ga, go, gg = torch.ops.nlspn.propagate_backward(pred_init, dep, confidence, aff, offset, gamma,
                                                                pred_inter, aff_out, conf_out, g_pred, g_inter, kh,
                                                                kw, affinity, pre, clip)
        return (gp, None, gc if confidence is not None else None, ga, go if offset is not None else None,
                gg if affinity == "TGASS" else None) + (None,) * 6

    torch.library.register_autograd("nlspn::propagate", bwd_propagate, setup_context=setup_propagate)

    def setup_step(ctx, inputs, output):
        feat, confidence, dep, aff, offset, kh, kw, raw_offsets, preserve_input, always_clip = inputs
        # (the inserted layout has no backward: raised in bwd_step, as _PropStepFn.backward
        # does, so a forward with grad mode on still runs)
        ctx.inserted = offset is not None and not raw_offsets
        ctx.save_for_backward(feat, confidence, dep, aff, offset)
        ctx.cfg = (kh, kw, preserve_input, always_clip)

    def bwd_step(ctx, g_out):
        if ctx.inserted:
            raise NotImplementedError("nlspn::prop_step's backward takes raw_offsets=True (B, 2K, H, W) offsets")
        feat, confidence, dep, aff, offset = ctx.saved_tensors
        gf, gc, ga, go = torch.ops.nlspn.prop_step_backward(feat, confidence, dep, aff, offset, g_out, *ctx.cfg)
        return (gf, gc if confidence is not None else None, None, ga, go if offset is not None else None) + \
            (None,) * 5

    torch.library.register_autograd("nlspn::prop_step", bwd_step, setup_context=setup_step)

    def setup_affnorm(ctx, inputs, output):
        aff, gamma, kind = inputs
        ctx.save_for_backward(aff, gamma)
        ctx.kind = kind

    def bwd_affnorm(ctx, g_out):
        aff, gamma = ctx.saved_tensors
        g_raw, g_gamma = torch.ops.nlspn.affinity_normalization_backward(aff, gamma, g_out, ctx.kind)
        return g_raw, g_gamma if ctx.kind == "TGASS" else None, None

    torch.library.register_autograd("nlspn::affinity_normalization", bwd_affnorm, setup_context=setup_affnorm)

    def setup_mdcn(ctx, inputs, output):
        inp, weight, bias, offset, mask = inputs[:5]
        ctx.save_for_backward(inp, weight, bias, offset, mask)
        ctx.ints = tuple(inputs[5:])

    def bwd_mdcn(ctx, g_out):
        inp, weight, bias, offset, mask = ctx.saved_tensors
        b = bias if bias is not None else weight.new_zeros((weight.shape[0],))
        gi, goff, gm, gw, gb = torch.ops.nlspn.modulated_deform_conv_backward(inp, weight, b, offset, mask,
                                                                             g_out.contiguous(), *ctx.ints)
        return (gi, gw, gb if bias is not None else None, goff, gm) + (None,) * 11

    torch.library.register_autograd("nlspn::modulated_deform_conv_forward", bwd_mdcn, setup_context=setup_mdcn)
