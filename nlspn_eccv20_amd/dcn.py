"""Seam 2 of the drop-in: a `DCN`-compatible module backed by the HIP library.

Reference: the pybind module `DCN` (src/model/deformconv/src/vision.cpp:6-13) whose
`modulated_deform_conv_forward` NLSPN reaches through
src/model/modulated_deform_conv_func.py:13,26 (ModulatedDeformConvFunction).
Installing this module as `DCN` (``sys.modules['DCN'] = nlspn_eccv20_amd.dcn``)
lets the unmodified reference nlspnmodel.py run its offset branch on MI355X.
Forward and backward (vision.cpp:9-10) are native HIP kernels (nlspn_mdcn.h).
"""
from __future__ import annotations

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable
from torch.nn.modules.utils import _pair

from . import _lib
from .propagation import _cuda, _ptr, _stream

_DCN_DTYPES = {torch.float32: _lib.DTYPE_F32, torch.float16: _lib.DTYPE_F16, torch.float64: _lib.DTYPE_F64}


def _dcn_dtype(t: torch.Tensor, backward: bool = False) -> int:
    """float32 / float64 (the reference's AT_DISPATCH_FLOATING_TYPES, .cu:93 / .cu:221);
    float16 storage for the forward (float arithmetic)."""
    if t.dtype not in _DCN_DTYPES or (backward and t.dtype == torch.float16):
        raise NotImplementedError(f"modulated_deform_conv_{'backward' if backward else 'forward'}: "
                                  f"dtype {t.dtype} is not supported")
    return _DCN_DTYPES[t.dtype]

__all__ = ["modulated_deform_conv_forward", "modulated_deform_conv_backward", "ModulatedDeformConvFunction"]


def modulated_deform_conv_forward(input, weight, bias, offset, mask, kernel_h, kernel_w, stride_h, stride_w,
                                  pad_h, pad_w, dilation_h, dilation_w, group, deformable_group, im2col_step):
    """Same signature and checks as modulated_deform_conv_cuda_forward
    (modulated_deform_conv_cuda.cu:19-121); returns (B, Cout, Ho, Wo).  im2col_step is
    accepted for signature compatibility; there is no columns buffer to chunk."""
    if not input.is_contiguous():
        raise RuntimeError("input tensor has to be contiguous")
    if not weight.is_contiguous():
        raise RuntimeError("weight tensor has to be contiguous")
    for n, t in (("input", input), ("weight", weight), ("bias", bias), ("offset", offset), ("mask", mask)):
        _cuda(n, t)
    B, C, H, W = input.shape
    Cout, Ckern, kh_, kw_ = weight.shape
    if kh_ != kernel_h or kw_ != kernel_w:
        raise RuntimeError(f"Input shape and kernel shape wont match: ({kernel_h} x {kernel_w} vs {kh_} x {kw_}).")
    if C != Ckern * group:
        raise RuntimeError(f"Input shape and kernel channels wont match: ({C} vs {Ckern * group}).")
    Ho = (H + 2 * pad_h - (dilation_h * (kernel_h - 1) + 1)) // stride_h + 1
    Wo = (W + 2 * pad_w - (dilation_w * (kernel_w - 1) + 1)) // stride_w + 1
    KK = kernel_h * kernel_w
    if tuple(offset.shape) != (B, 2 * deformable_group * KK, Ho, Wo):
        raise RuntimeError(f"offset has shape {tuple(offset.shape)}, expected {(B, 2 * deformable_group * KK, Ho, Wo)}")
    if tuple(mask.shape) != (B, deformable_group * KK, Ho, Wo):
        raise RuntimeError(f"mask has shape {tuple(mask.shape)}, expected {(B, deformable_group * KK, Ho, Wo)}")
    dt = input.dtype
    offset, mask, weight = offset.contiguous(), mask.contiguous(), weight.contiguous()
    if bias is not None:
        bias = bias.contiguous()
    for n, t in (("weight", weight), ("bias", bias), ("offset", offset), ("mask", mask)):
        if t is not None and t.dtype != dt:
            raise RuntimeError(f"{n} dtype {t.dtype} differs from input dtype {dt}")
    out = torch.empty((B, Cout, Ho, Wo), dtype=dt, device=input.device)
    with torch.cuda.device(input.device):
        _lib.check(_lib.get().nlspn_mdcn_forward(
            _dcn_dtype(input), _ptr(input), _ptr(weight), _ptr(bias), _ptr(offset), _ptr(mask), _ptr(out),
            B, C, H, W, Cout, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
            group, deformable_group, _stream(input.device)))
    return out


def modulated_deform_conv_backward(input, weight, bias, offset, mask, grad_output, kernel_h, kernel_w, stride_h,
                                   stride_w, pad_h, pad_w, dilation_h, dilation_w, group, deformable_group,
                                   im2col_step):
    """Same signature, checks and return list as modulated_deform_conv_cuda_backward
    (modulated_deform_conv_cuda.cu:124-280): [grad_input, grad_offset, grad_mask,
    grad_weight, grad_bias].  float32 or float64, as the reference dispatches
    (.cu:221).  Like the reference's col2im call (.cuh:371) grad_input uses pad_h for
    the width padding too (identical for square padding)."""
    if not input.is_contiguous():
        raise RuntimeError("input tensor has to be contiguous")
    if not weight.is_contiguous():
        raise RuntimeError("weight tensor has to be contiguous")
    for n, t in (("input", input), ("weight", weight), ("bias", bias), ("offset", offset), ("mask", mask),
                 ("grad_output", grad_output)):
        _cuda(n, t)
    dt = _dcn_dtype(input, backward=True)
    for n, t in (("weight", weight), ("bias", bias), ("offset", offset), ("mask", mask), ("grad_output", grad_output)):
        if t is not None and t.dtype != input.dtype:
            raise RuntimeError(f"{n} dtype {t.dtype} differs from input dtype {input.dtype}")
    B, C, H, W = input.shape
    Cout, Ckern, kh_, kw_ = weight.shape
    if (C % group) != 0 or (Cout % group) != 0:
        raise RuntimeError(f"channels({C}) and channels_out({Cout}) must divide group({group})")
    if kh_ != kernel_h or kw_ != kernel_w:
        raise RuntimeError(f"Input shape and kernel shape wont match: ({kernel_h} x {kernel_w} vs {kh_} x {kw_}).")
    if C != Ckern * group:
        raise RuntimeError(f"Input shape and kernel channels wont match: ({C} vs {Ckern * group}).")
    Ho = (H + 2 * pad_h - (dilation_h * (kernel_h - 1) + 1)) // stride_h + 1
    Wo = (W + 2 * pad_w - (dilation_w * (kernel_w - 1) + 1)) // stride_w + 1
    if grad_output.shape[0] != B:
        raise RuntimeError(f"Input shape and grad_out batch wont match: ({B} vs {grad_output.shape[0]}).")
    if grad_output.shape[1] != Cout:
        raise RuntimeError(f"Input shape and grad_out channels_out wont match: ({Cout} vs {grad_output.shape[1]}).")
    if tuple(grad_output.shape[2:]) != (Ho, Wo):
        raise RuntimeError(f"Input shape and grad_out shape wont match: ({Ho} x {Wo} vs "
                           f"{grad_output.shape[2]} x {grad_output.shape[3]}).")
    offset, mask, grad_output = offset.contiguous(), mask.contiguous(), grad_output.contiguous()
    grad_input = torch.empty_like(input)
    grad_offset = torch.empty_like(offset)
    grad_mask = torch.empty_like(mask)
    grad_weight = torch.empty_like(weight)
    grad_bias = torch.empty_like(bias) if bias is not None else None
    with torch.cuda.device(input.device):
        _lib.check(_lib.get().nlspn_mdcn_backward(
            dt, _ptr(input), _ptr(weight), _ptr(offset), _ptr(mask), _ptr(grad_output),
            _ptr(grad_input), _ptr(grad_offset), _ptr(grad_mask), _ptr(grad_weight), _ptr(grad_bias),
            B, C, H, W, Cout, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
            group, deformable_group, _stream(input.device)))
    return [grad_input, grad_offset, grad_mask, grad_weight, grad_bias]


class ModulatedDeformConvFunction(Function):
    """Mirror of src/model/modulated_deform_conv_func.py:15-56 (same apply() signature)."""

    @staticmethod
    def forward(ctx, input, offset, mask, weight, bias, stride, padding, dilation, groups, deformable_groups,
                im2col_step):
        ctx.stride = _pair(stride)
        ctx.padding = _pair(padding)
        ctx.dilation = _pair(dilation)
        ctx.kernel_size = _pair(weight.shape[2:4])
        ctx.groups = groups
        ctx.deformable_groups = deformable_groups
        ctx.im2col_step = im2col_step
        output = modulated_deform_conv_forward(
            input, weight, bias, offset, mask, ctx.kernel_size[0], ctx.kernel_size[1], ctx.stride[0], ctx.stride[1],
            ctx.padding[0], ctx.padding[1], ctx.dilation[0], ctx.dilation[1], ctx.groups, ctx.deformable_groups,
            ctx.im2col_step)
        ctx.save_for_backward(input, offset, mask, weight, bias)
        return output

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        input, offset, mask, weight, bias = ctx.saved_tensors
        grad_input, grad_offset, grad_mask, grad_weight, grad_bias = modulated_deform_conv_backward(
            input, weight, bias, offset, mask, grad_output, ctx.kernel_size[0], ctx.kernel_size[1], ctx.stride[0],
            ctx.stride[1], ctx.padding[0], ctx.padding[1], ctx.dilation[0], ctx.dilation[1], ctx.groups,
            ctx.deformable_groups, ctx.im2col_step)
        return grad_input, grad_offset, grad_mask, grad_weight, grad_bias, None, None, None, None, None, None

