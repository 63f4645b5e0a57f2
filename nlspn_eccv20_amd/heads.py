"""Head epilogue on the HIP kernel: the decoder's last three 3x3
convolutions as one kernel.

Reference: src/model/nlspnmodel.py:296-315 —
    pred_init  = id_dec0(cat(id_fd1, fe1))        ReLU      (:297, id_dec0 :68)
    off_aff    = off_aff_dec0(cat(off_aff_fd1, fe1))         (:301, off_aff_dec0 :74/:76)
    confidence = cf_dec0(cat(cf_fd1, fe1))        Sigmoid   (:313, cf_dec0 :83-86)
``head_epilogue`` reads fe1 and the three decoder outputs in place (no concatenated
copies) and computes all three convolutions with bias and activation in one launch
(``nlspn_head_epilogue``, ``csrc/nlspn_heads.h``): f32 operands on the matrix cores,
exact f32 products, f32 accumulation.  Inference only (no autograd formula): the model
calls it when gradients are off; training keeps the torch convolutions.

The three convolutions' weights are packed once per weight version into the kernel's
layout (``nlspn_head_pack_weights``) and cached on the module.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib

__all__ = ["head_epilogue", "head_epilogue_prologue", "HeadWeights"]


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _conv_of(m):
    """The nn.Conv2d of a head (a bare conv, or the first layer of conv_bn_relu /
    cf_dec0's Sequential)."""
    if m is None or isinstance(m, nn.Conv2d):
        return m
    return m[0]


class _Packed:
    __slots__ = ("key", "wm", "wv", "bias", "C", "nout", "keep")


class HeadWeights:
    """The packed weights of (off_aff_dec0, id_dec0, cf_dec0), one entry per device,
    rebuilt when any of the convolutions' parameters change (storage pointer or tensor
    version counter).  An entry is never mutated after it is built, so DataParallel
    replicas sharing this cache from their threads each get their own device's entry."""

    def __init__(self):
        self._entries = {}

    @staticmethod
    def _check(conv, name, nout=None):
        if conv is None:
            return
        if conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1) or conv.dilation != (1, 1) \
                or conv.groups != 1 or conv.bias is None:
            raise RuntimeError(f"{name} must be a 3x3 / stride 1 / pad 1 convolution with bias (conv_bn_relu(..., "
                               "bn=False), nlspnmodel.py:68-86)")
        if nout is not None and conv.out_channels != nout:
            raise RuntimeError(f"{name} must have {nout} output channel(s), has {conv.out_channels}")
        if conv.weight.dtype != torch.float32 or not conv.weight.is_cuda:
            raise RuntimeError(f"{name} weights must be float32 CUDA tensors")

    def get(self, oa, idc, cfc) -> _Packed:
        self._check(oa, "off_aff_dec0")
        self._check(idc, "id_dec0", 1)
        self._check(cfc, "cf_dec0", 1)
        C2 = oa.in_channels
        for c, n in ((idc, "id_dec0"), (cfc, "cf_dec0")):
            if c is not None and c.in_channels != C2:
                raise RuntimeError(f"{n} must read {C2} channels like off_aff_dec0, reads {c.in_channels}")
        params = [t for c in (oa, idc, cfc) if c is not None for t in (c.weight, c.bias)]
        key = (tuple((t.data_ptr(), t._version) for t in params), idc is None, cfc is None)
        dev = oa.weight.device
        e = self._entries.get(dev)
        if e is not None and e.key == key:
            return e
        C, nout = C2 // 2, oa.out_channels
        lib = _lib.get()
        nm, nv, nb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(lib.nlspn_head_packed_size(C, nout, ctypes.byref(nm), ctypes.byref(nv), ctypes.byref(nb)))
        e = _Packed()
        e.wm = torch.empty(nm.value, dtype=torch.float32, device=dev)
        e.wv = torch.empty(nv.value, dtype=torch.float32, device=dev)
        e.bias = torch.empty(nb.value, dtype=torch.float32, device=dev)
        w = lambda c: None if c is None else c.weight.detach().contiguous()  # noqa: E731
        b = lambda c: None if c is None else c.bias.detach().contiguous()  # noqa: E731
        e.keep = [w(oa), b(oa), w(idc), b(idc), w(cfc), b(cfc)]  # alive until the pack kernel has run
        with torch.cuda.device(dev):
            _lib.check(lib.nlspn_head_pack_weights(*[_p(t) for t in e.keep], _p(e.wm), _p(e.wv), _p(e.bias),
                                                   C, nout, _stream(dev)))
        e.key, e.C, e.nout = key, C, nout
        self._entries[dev] = e
        return e


def head_epilogue(fe1, off_aff_fd1, off_aff_dec0, id_fd1=None, id_dec0=None, cf_fd1=None, cf_dec0=None,
                  weights: HeadWeights | None = None):
    """(pred_init, off_aff, confidence) of nlspnmodel.py:297-315 from the decoder outputs.
    ``id_fd1``/``id_dec0`` and ``cf_fd1``/``cf_dec0`` may be None (that head is skipped
    and None returned for it)."""
    oa, idc, cfc = _conv_of(off_aff_dec0), _conv_of(id_dec0), _conv_of(cf_dec0)
    if (id_fd1 is None) != (idc is None) or (cf_fd1 is None) != (cfc is None):
        raise RuntimeError("each head needs both its decoder output and its convolution")
    weights = (weights or HeadWeights()).get(oa, idc, cfc)  # this device's packed entry
    srcs = [fe1, off_aff_fd1, id_fd1, cf_fd1]
    B, C, H, W = fe1.shape
    if C != weights.C:
        raise RuntimeError(f"fe1 has {C} channels, the head convolutions expect {weights.C} + {weights.C}")
    for n, t in zip(("fe1", "off_aff_fd1", "id_fd1", "cf_fd1"), srcs):
        if t is None:
            continue
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError(f"{n} must be a float32 CUDA tensor")
        if tuple(t.shape) != (B, C, H, W):
            raise RuntimeError(f"{n} must be {(B, C, H, W)} (the _concat crop is done by the caller), got "
                               f"{tuple(t.shape)}")
    srcs = [None if t is None else t.contiguous() for t in srcs]
    dev = fe1.device
    off_aff = torch.empty((B, weights.nout, H, W), dtype=torch.float32, device=dev)
    pred_init = torch.empty((B, 1, H, W), dtype=torch.float32, device=dev) if id_fd1 is not None else None
    conf = torch.empty((B, 1, H, W), dtype=torch.float32, device=dev) if cf_fd1 is not None else None
    with torch.cuda.device(dev):
        _lib.check(_lib.get().nlspn_head_epilogue(
            _lib.DTYPE_F32, *[_p(t) for t in srcs], _p(weights.wm), _p(weights.wv), _p(weights.bias), _p(off_aff),
            _p(pred_init), _p(conf), B, C, H, W, weights.nout, _stream(dev)))
    return pred_init, off_aff, conf


def head_epilogue_prologue(fe1, off_aff_fd1, off_aff_dec0, id_fd1, id_dec0, dep, gamma, affinity="TGASS",
                           cf_fd1=None, cf_dec0=None, preserve_input=True, always_clip=False,
                           weights: HeadWeights | None = None) -> dict:
    """The three head convolutions with the propagation prologue fused into their
    epilogue (3x3, K = 8, offsets on; nlspnmodel.py:297-348): returns {'pred_init',
    'offset' (_off_insert, :324), 'aff' (normalised + reference tap, :325),
    'confidence' (blended, :328-334, or None), 'p0' (iteration 1's input, :341-348)} —
    what nlspn_propagate's step 1 would produce from the raw head outputs, bit for bit.
    Feed them to propagation.propagate_normalized."""
    from .propagation import _gamma_f32
    oa, idc, cfc = _conv_of(off_aff_dec0), _conv_of(id_dec0), _conv_of(cf_dec0)
    if (cf_fd1 is None) != (cfc is None) or id_fd1 is None or idc is None:
        raise RuntimeError("the fused prologue needs id_fd1/id_dec0, and cf_fd1 with cf_dec0")
    if oa.out_channels != 24:
        raise RuntimeError("the fused prologue is the 3x3 / K=8 / offset geometry (off_aff_dec0 -> 24 channels)")
    from . import _lib as L
    if affinity not in L.AFF_KINDS:
        raise NotImplementedError(affinity)
    weights = (weights or HeadWeights()).get(oa, idc, cfc)
    B, C, H, W = fe1.shape
    srcs = [fe1, off_aff_fd1, id_fd1, cf_fd1]
    for n, t in zip(("fe1", "off_aff_fd1", "id_fd1", "cf_fd1"), srcs):
        if t is None:
            continue
        if not t.is_cuda or t.dtype != torch.float32 or tuple(t.shape) != (B, C, H, W):
            raise RuntimeError(f"{n} must be a float32 CUDA tensor of shape {(B, C, H, W)}")
    if preserve_input and (dep is None or tuple(dep.shape) != (B, 1, H, W)):
        raise RuntimeError("preserve_input requires dep of shape (B, 1, H, W)")
    srcs = [None if t is None else t.contiguous() for t in srcs]
    dep = None if dep is None else dep.contiguous().float()
    g = _gamma_f32(gamma)
    dev = fe1.device
    e = lambda c: torch.empty((B, c, H, W), dtype=torch.float32, device=dev)  # noqa: E731
    out = {"pred_init": e(1), "offset": e(18), "aff": e(9), "confidence": e(1) if cf_fd1 is not None else None,
           "p0": e(1)}
    flags = (L.PRESERVE_INPUT if preserve_input else 0) | (L.ALWAYS_CLIP if always_clip else 0)
    with torch.cuda.device(dev):
        L.check(L.get().nlspn_head_epilogue_prologue(
            L.DTYPE_F32, *[_p(t) for t in srcs], _p(weights.wm), _p(weights.wv), _p(weights.bias), _p(dep), _p(g),
            _p(out["pred_init"]), _p(out["confidence"]), _p(out["aff"]), _p(out["offset"]), _p(out["p0"]),
            B, C, H, W, 3, 3, L.AFF_KINDS[affinity], flags, _stream(dev)))
    return out
