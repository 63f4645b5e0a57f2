"""MI355X-native NLSPN propagation — host-side mirror of the reference interface.

Reference (XJTUXYC/NLSPN_ECCV20, src/model/nlspnmodel.py):
  _affinity_normalization :179-201   -> affinity_normalization()
  _aff_insert             :261-269   -> (fused into affinity_normalization)
  _off_insert             :252-259   -> off_insert()
  _propagate_once         :203-226   -> prop_step() (fused with :351 and :355-361)
  forward, propagation    :317-383   -> propagate() / NLSPNPropagation.forward()

Every call goes through the C ABI in include/nlspn_prop.h (HIP kernels for
gfx950); there is no CPU path.  Tensors are NCHW with contiguous (H, W) planes;
per-batch strides are passed through, so the (B, 3K, H, W) head output can be
sliced into offsets/affinities without a copy (nlspnmodel.py:304-305).
Computation is fp32; storage may be fp32 or fp16.

propagate() is differentiable (float32 storage): its backward is the native
nlspn_propagate_backward (DCN col2im/col2im_coord + the autograd of the blends,
clamps and affinity normalisation), giving gradients for pred_init, confidence,
the raw affinity, the raw offsets and gamma.  prop_step() and
affinity_normalization() are inference building blocks.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import _lib

__all__ = [
    "affinity_normalization", "off_insert", "prop_step", "propagate", "PropagationPlan",
    "NLSPNPropagation", "kernel_geometry",
]


# ----------------------------------------------------------------- helpers
def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return _lib.DTYPE_F32
    if t.dtype == torch.float16:
        return _lib.DTYPE_F16
    raise TypeError(f"NLSPN propagation supports float32 and float16 storage, got {t.dtype}")


def _cuda(name: str, t: Optional[torch.Tensor]) -> None:
    # modulated_deform_conv_cuda.cu:42-46 ("... must be a CUDA tensor")
    if t is not None and not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _planes(name: str, t: torch.Tensor, B: int, C: Optional[int], H: int, W: int) -> int:
    """Check (B, C, H, W) with contiguous H*W planes, consecutive within a batch item;
    return the batch stride in elements."""
    if t.dim() != 4 or t.shape[0] != B or tuple(t.shape[2:]) != (H, W) or (C is not None and t.shape[1] != C):
        want = f"({B}, {C if C is not None else '*'}, {H}, {W})"
        raise RuntimeError(f"{name} has shape {tuple(t.shape)}, expected {want}")
    if t.stride(3) != 1 or (H > 1 and t.stride(2) != W) or (t.shape[1] > 1 and t.stride(1) != H * W):
        raise RuntimeError(f"{name} tensor has to have contiguous H*W planes")
    return t.stride(0) if B > 1 else t.shape[1] * H * W


def kernel_geometry(prop_kernel) -> Tuple[int, int]:
    """prop_kernel int k -> (k, k); or an explicit (kh, kw).  Odd sizes only
    (nlspnmodel.py:29-30).  K = kh*kw - 1 neighbours."""
    kh, kw = (prop_kernel, prop_kernel) if isinstance(prop_kernel, int) else tuple(prop_kernel)
    if kh % 2 != 1 or kw % 2 != 1:
        raise AssertionError(f"only odd kernel is supported but k_f = {prop_kernel}")
    return int(kh), int(kw)


_OPS = None


def _torch_ops():
    """torch.ops.nlspn when the operator layer (libnlspn_torch.so) is built, else None:
    the ops run the same kernels with ~2.5x less host cost per call than ctypes
    (tools/op_overhead.py), which matters where a call is issued per iteration (GRU mode)."""
    global _OPS
    if _OPS is None:
        from . import ops
        _OPS = torch.ops.nlspn if ops.available() else False
    return _OPS or None


def _gamma_f32(gamma) -> torch.Tensor:
    if not torch.is_tensor(gamma):
        raise TypeError("gamma must be a device tensor (aff_scale_const)")
    g = gamma.detach().reshape(-1)[:1]
    return g if g.dtype == torch.float32 else g.float()


# -------------------------------------------------------------- functional ops
def _affinity_normalization(aff: torch.Tensor, gamma: torch.Tensor, kind: str) -> torch.Tensor:
    _cuda("aff", aff)
    if kind not in _lib.AFF_KINDS:
        raise NotImplementedError(kind)
    B, K, H, W = aff.shape
    bs = _planes("aff", aff, B, K, H, W)
    g = _gamma_f32(gamma)
    out = torch.empty((B, K + 1, H, W), dtype=aff.dtype, device=aff.device)
    with torch.cuda.device(aff.device):
        _lib.check(_lib.get().nlspn_affinity_normalize(
            _dtype_code(aff), _ptr(aff), bs, _ptr(g), _ptr(out), B, K, H, W, _lib.AFF_KINDS[kind],
            _stream(aff.device)))
    return out


class _AffNormFn(torch.autograd.Function):
    """Autograd node for affinity_normalization; backward = nlspn_affinity_normalize_backward."""

    @staticmethod
    def forward(ctx, aff, gamma, kind):
        ctx.kind = kind
        ctx.save_for_backward(aff, gamma)
        return _affinity_normalization(aff, gamma, kind)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_out):
        aff, gamma = ctx.saved_tensors
        g_raw, g_gamma = _affnorm_backward(aff, gamma, g_out, ctx.kind, ctx.needs_input_grad[1])
        return g_raw, g_gamma, None


def _affnorm_backward(aff, gamma, g_out, kind, want_gamma=True):
    """nlspn_affinity_normalize_backward: gradients of the (K+1)-tap normalised affinity
    with respect to the raw taps and (TGASS, want_gamma) gamma (else None)."""
    if aff.dtype != torch.float32:
        raise NotImplementedError("the affinity-normalisation backward is implemented for float32 storage")
    B, K, H, W = aff.shape
    f32 = dict(dtype=torch.float32, device=aff.device)
    g_out = g_out.contiguous()
    g_raw = torch.empty((B, K, H, W), **f32)
    want_g = kind == "TGASS" and want_gamma
    g_gamma = torch.empty(1, **f32) if want_g else None
    lib = _lib.get()
    ws = torch.empty(max(1, lib.nlspn_affinity_normalize_backward_workspace_bytes(B, K, H, W) // 4), **f32)
    with torch.cuda.device(aff.device):
        _lib.check(lib.nlspn_affinity_normalize_backward(
            _lib.DTYPE_F32, _ptr(aff), _planes("aff", aff, B, K, H, W), _ptr(_gamma_f32(gamma)), _ptr(g_out),
            _ptr(g_raw), _ptr(g_gamma), _ptr(ws), B, K, H, W, _lib.AFF_KINDS[kind], _stream(aff.device)))
    if g_gamma is not None:
        g_gamma = g_gamma.reshape(gamma.shape).to(gamma.dtype)
    return g_raw, g_gamma


def affinity_normalization(aff: torch.Tensor, gamma: torch.Tensor, kind: str = "TGASS") -> torch.Tensor:
    """NLSPNModel._affinity_normalization + _aff_insert (nlspnmodel.py:179-201, :261-269).
    aff (B, K, H, W) raw -> (B, K+1, H, W), reference tap at K//2.  Differentiable
    (float32) in aff and, for TGASS, gamma."""
    if torch.is_grad_enabled() and (aff.requires_grad or (torch.is_tensor(gamma) and gamma.requires_grad)):
        return _AffNormFn.apply(aff, gamma, kind)
    top = _torch_ops()
    if top is not None and aff.is_cuda and torch.is_tensor(gamma) and gamma.is_cuda:
        return top.affinity_normalization(aff, gamma, kind)
    return _affinity_normalization(aff, gamma, kind)


def off_insert(offset: torch.Tensor) -> torch.Tensor:
    """NLSPNModel._off_insert (nlspnmodel.py:252-259): (B, 2K, H, W) -> (B, 2(K+1), H, W)
    with a zero (dh, dw) pair at tap K//2.  A layout conversion, kept in torch."""
    B, K2, H, W = offset.shape
    K = K2 // 2
    o = offset.reshape(B, K, 2, H, W)
    z = torch.zeros((B, 1, 2, H, W), dtype=offset.dtype, device=offset.device)
    return torch.cat([o[:, :K // 2], z, o[:, K // 2:]], 1).reshape(B, -1, H, W)


def _prop_step(feat, confidence, dep, aff, offset, kernel, offset_layout, preserve_input, always_clip, out=None,
               pred_out=None):
    kh, kw = kernel_geometry(kernel)
    K = kh * kw - 1
    for n, t in (("feat", feat), ("confidence", confidence), ("dep", dep), ("aff", aff), ("offset", offset)):
        _cuda(n, t)
    B, _, H, W = feat.shape
    _planes("feat", feat, B, 1, H, W)
    if not feat.is_contiguous():
        raise RuntimeError("input tensor has to be contiguous")
    for n, t in (("confidence", confidence), ("dep", dep)):
        if t is not None:
            _planes(n, t, B, 1, H, W)
            if t.dtype != feat.dtype or not t.is_contiguous():
                raise RuntimeError(f"{n} must be contiguous with feat's dtype")
    if preserve_input and dep is None:
        raise RuntimeError("preserve_input requires dep")
    abs_ = _planes("aff", aff, B, K + 1, H, W)
    layout = _lib.OFF_RAW if offset_layout == "raw" else _lib.OFF_INSERTED
    obs = 0
    if offset is not None:
        obs = _planes("offset", offset, B, 2 * K if layout == _lib.OFF_RAW else 2 * (K + 1), H, W)
    if out is None:
        out = torch.empty_like(feat)
    flags = (_lib.PRESERVE_INPUT if preserve_input else 0) | (_lib.ALWAYS_CLIP if always_clip else 0)
    with torch.cuda.device(feat.device):
        _lib.check(_lib.get().nlspn_prop_step(
            _dtype_code(feat), _ptr(feat), _ptr(confidence), _ptr(dep), _ptr(aff), abs_, _ptr(offset), obs,
            layout, _ptr(out), _ptr(pred_out), B, H, W, kh, kw, flags, _stream(feat.device)))
    return out


class _PropStepFn(torch.autograd.Function):
    """Autograd node for one prop_step; backward = nlspn_prop_step_backward (float32,
    raw offset layout).  dep receives no gradient (the reference's sparse input)."""

    @staticmethod
    def forward(ctx, feat, confidence, dep, aff, offset, kernel, offset_layout, preserve_input, always_clip):
        ctx.cfg = (kernel_geometry(kernel), offset_layout, preserve_input, always_clip)
        ctx.save_for_backward(feat, confidence, dep, aff, offset)
        return _prop_step(feat, confidence, dep, aff, offset, kernel, offset_layout, preserve_input, always_clip)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_out):
        feat, conf, dep, aff, off = ctx.saved_tensors
        (kh, kw), layout, preserve, clip = ctx.cfg
        if off is not None and layout != "raw":
            raise NotImplementedError("the prop_step backward takes offset_layout='raw' (B, 2K, H, W) offsets")
        g_feat, g_conf, g_aff, g_off = _step_backward(feat, conf, dep, aff, off, g_out, kh, kw, preserve, clip)
        return g_feat, g_conf, None, g_aff, g_off, None, None, None, None


def _step_backward(feat, conf, dep, aff, off, g_out, kh, kw, preserve, clip):
    """nlspn_prop_step_backward: gradients of one iteration with respect to feat,
    confidence, the normalised (K+1)-tap affinity (tap K/2 zero: recomputed in-kernel as
    1 - sum) and the raw offsets (None where the input is absent)."""
    if feat.dtype != torch.float32:
        raise NotImplementedError("the prop_step backward is implemented for float32 storage")
    B, _, H, W = feat.shape
    K = kh * kw - 1
    f32 = dict(dtype=torch.float32, device=feat.device)
    g_feat = torch.empty((B, 1, H, W), **f32)
    g_conf = torch.empty((B, 1, H, W), **f32) if conf is not None else None
    g_aff = torch.empty((B, K + 1, H, W), **f32)
    g_off = torch.empty((B, 2 * K, H, W), **f32) if off is not None else None
    lib = _lib.get()
    ws = torch.empty(lib.nlspn_prop_step_backward_workspace_bytes(B, H, W) // 4, **f32)
    flags = (_lib.PRESERVE_INPUT if preserve else 0) | (_lib.ALWAYS_CLIP if clip else 0)
    with torch.cuda.device(feat.device):
        _lib.check(lib.nlspn_prop_step_backward(
            _lib.DTYPE_F32, _ptr(feat), _ptr(conf), _ptr(dep), _ptr(aff), _planes("aff", aff, B, K + 1, H, W),
            _ptr(off), _planes("offset", off, B, 2 * K, H, W) if off is not None else 0,
            _ptr(g_out.contiguous()), _ptr(g_feat), _ptr(g_conf), _ptr(g_aff), _ptr(g_off), _ptr(ws),
            B, H, W, kh, kw, flags, _stream(feat.device)))
    return g_feat, g_conf, g_aff, g_off


def prop_step(feat: torch.Tensor, confidence: Optional[torch.Tensor], dep: Optional[torch.Tensor],
              aff: torch.Tensor, offset: Optional[torch.Tensor] = None, *, kernel=(3, 3),
              offset_layout: str = "inserted", preserve_input: bool = True, always_clip: bool = False,
              out: Optional[torch.Tensor] = None, pred_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One fused iteration (nlspnmodel.py:350-361): out = _propagate_once(feat*confidence,
    offset, aff), then the preserve-input blend with dep and the optional clamp.

    aff: normalised (B, K+1, H, W) (the output of affinity_normalization; its tap K//2 is
    recomputed in-kernel as 1 - sum of the others).  offset: (B, 2(K+1), H, W) inserted
    layout or (B, 2K, H, W) with offset_layout="raw"; None = no-offset branch (3x3 replicate).
    Differentiable (float32, raw offsets) in feat, confidence, aff and offset when called
    without out/pred_out.
    """
    if (out is None and pred_out is None and torch.is_grad_enabled()
            and any(t is not None and t.requires_grad for t in (feat, confidence, aff, offset))):
        return _PropStepFn.apply(feat, confidence, dep, aff, offset, kernel, offset_layout, preserve_input,
                                 always_clip)
    top = _torch_ops()
    if top is not None and out is None and pred_out is None and feat.is_cuda:
        kh, kw = kernel_geometry(kernel)
        return top.prop_step(feat, confidence, dep, aff, offset, kh, kw, offset_layout == "raw", preserve_input,
                             always_clip)
    return _prop_step(feat, confidence, dep, aff, offset, kernel, offset_layout, preserve_input, always_clip, out,
                      pred_out)


def _alloc_outputs(pred_init, K, T, with_off, with_conf):
    B, _, H, W = pred_init.shape
    kw_ = dict(dtype=pred_init.dtype, device=pred_init.device)
    return {
        "pred_inter": torch.empty((T, B, 1, H, W), **kw_),
        "pred": torch.empty((B, 1, H, W), **kw_),
        "aff": torch.empty((B, K + 1, H, W), **kw_),
        "offset": torch.empty((B, 2 * (K + 1), H, W), **kw_) if with_off else None,
        "confidence": torch.empty((B, 1, H, W), **kw_) if with_conf else None,
        # sync words of the resident kernel (abort word, per-part placement words)
        "workspace": torch.empty(_lib.get().nlspn_workspace_bytes(_dtype_code(pred_init), B, H, W) // 4,
                                 dtype=torch.int32, device=pred_init.device),
    }


def _propagate_args(pred_init, dep, confidence, aff, offset, gamma, kernel, prop_time, affinity,
                    preserve_input, always_clip, outs):
    kh, kw = kernel_geometry(kernel)
    K = kh * kw - 1
    for n, t in (("pred_init", pred_init), ("dep", dep), ("confidence", confidence), ("aff", aff),
                 ("offset", offset), ("gamma", gamma)):
        _cuda(n, t)
    if affinity not in _lib.AFF_KINDS:
        raise NotImplementedError(affinity)
    B, C, H, W = pred_init.shape
    if C != 1:
        raise AssertionError("ch_f must equal pred_init.shape[1] == 1 (nlspnmodel.py:318)")
    _planes("pred_init", pred_init, B, 1, H, W)
    dt = pred_init.dtype
    for n, t in (("dep", dep), ("confidence", confidence)):
        if t is not None:
            _planes(n, t, B, 1, H, W)
            if not t.is_contiguous() or t.dtype != dt:
                raise RuntimeError(f"{n} must be contiguous with pred_init's dtype")
    if not pred_init.is_contiguous():
        raise RuntimeError("pred_init must be contiguous")
    if preserve_input and dep is None:
        raise RuntimeError("preserve_input requires dep")
    abs_ = _planes("aff", aff, B, K, H, W)
    obs = _planes("offset", offset, B, 2 * K, H, W) if offset is not None else 0
    if aff.dtype != dt or (offset is not None and offset.dtype != dt):
        raise RuntimeError("aff/offset must have pred_init's dtype")
    flags = (_lib.PRESERVE_INPUT if preserve_input else 0) | (_lib.ALWAYS_CLIP if always_clip else 0)
    g = _gamma_f32(gamma)
    args = (_dtype_code(pred_init), _ptr(pred_init), _ptr(dep), _ptr(confidence), _ptr(aff), abs_,
            _ptr(offset), obs, _ptr(g), _ptr(outs["pred_inter"]), _ptr(outs["pred"]), _ptr(outs["aff"]),
            _ptr(outs["offset"]), _ptr(outs["confidence"]), _ptr(outs["workspace"]),
            B, H, W, kh, kw, int(prop_time), _lib.AFF_KINDS[affinity], flags)
    return args, g


class _PropagateFn(torch.autograd.Function):
    """Autograd node for the whole propagation section.  Differentiable outputs:
    pred and pred_inter.  aff (normalised), offset (inserted) and confidence
    (blended) are returned for the output dict but marked non-differentiable."""

    @staticmethod
    def forward(ctx, pred_init, dep, confidence, aff, offset, gamma, prop_time, affinity, kernel, preserve_input,
                always_clip, return_offset, packed=None):
        # packed: the (B, 3K, H, W) head output `offset` and `aff` are slices of
        # (nlspnmodel.py:304-305); its gradient is then built in one buffer
        ctx.packed = packed is not None
        kh, kw = kernel_geometry(kernel)
        outs = _alloc_outputs(pred_init, kh * kw - 1, prop_time, offset is not None and return_offset,
                              confidence is not None)
        args, _ = _propagate_args(pred_init, dep, confidence, aff, offset, gamma, kernel, prop_time, affinity,
                                  preserve_input, always_clip, outs)
        with torch.cuda.device(pred_init.device):
            _lib.check_resident()  # an earlier resident launch that aborted raises here
            _lib.check(_lib.get().nlspn_propagate(*args, _stream(pred_init.device)))
        ctx.cfg = (kh, kw, int(prop_time), affinity, preserve_input, always_clip)
        # an unused output's gradient arrives as None, not as a zero-filled tensor: a loss
        # on `pred` alone then neither fills nor reads the (T, B, 1, H, W) pred_inter
        # gradient (the C ABI takes null grad_pred / grad_pred_inter)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(pred_init, dep, confidence, aff, offset, gamma, outs["pred_inter"], outs["aff"],
                              outs["confidence"])
        nd = [t for t in (outs["aff"], outs["offset"], outs["confidence"]) if t is not None]
        ctx.mark_non_differentiable(*nd)
        return outs["pred"], outs["pred_inter"], outs["aff"], outs["offset"], outs["confidence"]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_pred, g_inter, _g_aff, _g_off, _g_conf):
        pred_init, dep, conf, aff, off, gamma, pred_inter, aff_norm, conf_eff = ctx.saved_tensors
        g_pi, g_conf, g_aff, g_off, g_gamma, g_oa = _section_backward(
            pred_init, dep, conf, aff, off, gamma, pred_inter, aff_norm, conf_eff, g_pred, g_inter, *ctx.cfg,
            packed=ctx.packed)
        if ctx.packed:
            return (g_pi, None, g_conf, None, None, g_gamma) + (None,) * 6 + (g_oa,)
        return (g_pi, None, g_conf, g_aff, g_off, g_gamma) + (None,) * 7


def _section_backward(pred_init, dep, conf, aff, off, gamma, pred_inter, aff_norm, conf_eff, g_pred, g_inter,
                      kh, kw, T, affinity, preserve, clip, packed=False):
    """nlspn_propagate_backward: gradients of the section (pred, pred_inter) with respect
    to pred_init, confidence, the raw affinity, the raw offsets and gamma (None where the
    input is absent; g_gamma None unless TGASS).  packed: the affinity and offset
    gradients as slices of one (B, 3K, H, W) buffer, returned last (else None)."""
    if pred_init.dtype != torch.float32:
        raise NotImplementedError("the propagation backward is implemented for float32 storage")
    B, _, H, W = pred_init.shape
    K = kh * kw - 1
    dev = pred_init.device
    f32 = dict(dtype=torch.float32, device=dev)
    g_pred = None if g_pred is None else g_pred.contiguous()
    g_inter = None if g_inter is None else g_inter.contiguous()
    g_pi = torch.empty((B, 1, H, W), **f32)
    g_conf = torch.empty((B, 1, H, W), **f32) if conf is not None else None
    g_oa = None
    if packed:  # one (B, 3K, H, W) gradient: offsets in planes 0..2K-1, affinity after
        g_oa = torch.empty((B, 3 * K, H, W), **f32)
        g_off, g_aff, gbs = g_oa[:, :2 * K], g_oa[:, 2 * K:], 3 * K * H * W
    else:
        g_aff = torch.empty((B, K, H, W), **f32)
        g_off = torch.empty((B, 2 * K, H, W), **f32) if off is not None else None
        gbs = 0
    g_gamma = torch.zeros(1, **f32)
    lib = _lib.get()
    ws = torch.empty(lib.nlspn_backward_workspace_bytes(B, H, W, kh, kw) // 4, **f32)
    g = _gamma_f32(gamma)
    flags = (_lib.PRESERVE_INPUT if preserve else 0) | (_lib.ALWAYS_CLIP if clip else 0)
    abs_ = _planes("aff", aff, B, K, H, W)
    obs = _planes("offset", off, B, 2 * K, H, W) if off is not None else 0
    with torch.cuda.device(dev):
        _lib.check(lib.nlspn_propagate_backward(
            _lib.DTYPE_F32, _ptr(pred_init), _ptr(dep), _ptr(conf), _ptr(aff), abs_, _ptr(off), obs, _ptr(g),
            _ptr(pred_inter), _ptr(aff_norm), _ptr(conf_eff), _ptr(g_pred), _ptr(g_inter), _ptr(g_pi),
            _ptr(g_conf), _ptr(g_aff), gbs, _ptr(g_off), gbs, _ptr(g_gamma), _ptr(ws), B, H, W, kh, kw, T,
            _lib.AFF_KINDS[affinity], flags, _stream(dev)))
    g_gamma = g_gamma.reshape(gamma.shape).to(gamma.dtype) if affinity == "TGASS" else None
    return g_pi, g_conf, g_aff, g_off, g_gamma, g_oa


def _packed_head(aff, offset):
    """The contiguous (B, 3K, H, W) tensor that `offset` (planes 0..2K-1) and `aff`
    (planes 2K..3K-1) are slices of, when it requires grad (nlspnmodel.py:304-305 slice
    the head output so): autograd then gets ONE gradient for it instead of two
    zero-filled full-size ones summed.  None otherwise — in particular when either
    slice does not itself require grad (e.g. it was cut off under no_grad), or the
    slices' strides differ from the base's.  Note: the gradient then flows to the
    base directly, so hooks / retain_grad() registered on the two slices do not fire."""
    if offset is None or aff._base is None or offset._base is not aff._base:
        return None
    base = aff._base
    if not base.requires_grad or base.dim() != 4 or not base.is_contiguous() or base.dtype != torch.float32:
        return None
    # slices taken under no_grad report requires_grad but have no grad_fn: not in the graph
    if not (aff.requires_grad and offset.requires_grad) or aff.grad_fn is None or offset.grad_fn is None:
        return None
    if aff.stride() != base.stride() or offset.stride() != base.stride():
        return None
    B, K = aff.shape[0], aff.shape[1]
    HW = aff.shape[2] * aff.shape[3]
    es = base.element_size()
    if (tuple(base.shape) != (B, 3 * K, aff.shape[2], aff.shape[3]) or offset.data_ptr() != base.data_ptr()
            or aff.data_ptr() != base.data_ptr() + 2 * K * HW * es or offset.shape[1] != 2 * K):
        return None
    return base


def propagate(pred_init: torch.Tensor, dep: Optional[torch.Tensor], confidence: Optional[torch.Tensor],
              aff: torch.Tensor, offset: Optional[torch.Tensor], gamma: torch.Tensor, *, prop_time: int = 18,
              affinity: str = "TGASS", kernel=(3, 3), preserve_input: bool = True, always_clip: bool = False,
              return_offset: bool = True) -> dict:
    """The propagation section of NLSPNModel.forward (nlspnmodel.py:323-381), fused:
    prop_time launches on the current stream (the prologue rides in the first).

    aff: raw affinity (B, K, H, W); offset: raw offsets (B, 2K, H, W) or None;
    gamma: aff_scale_const (device tensor, read on the device).
    Returns {'pred', 'pred_inter' (list of prop_time (B,1,H,W) views), 'offset'
    (inserted, or None), 'aff' (normalised, K+1 taps), 'confidence' (blended, or None)}.
    Differentiable in pred_init, confidence, aff, offset and gamma when autograd is on.
    """
    packed = _packed_head(aff, offset) if torch.is_grad_enabled() else None
    pred, pred_inter, aff_o, off_o, conf_o = _PropagateFn.apply(
        pred_init, dep, confidence, aff, offset, gamma, prop_time, affinity, kernel, preserve_input, always_clip,
        return_offset, packed)
    return {"pred": pred, "pred_inter": list(pred_inter.unbind(0)), "offset": off_o, "aff": aff_o,
            "confidence": conf_o, "pred_inter_tensor": pred_inter}


def propagate_normalized(p0: torch.Tensor, dep: Optional[torch.Tensor], confidence: Optional[torch.Tensor],
                         aff: torch.Tensor, offset: torch.Tensor, prop_time: int = 18, kernel=3,
                         preserve_input: bool = True, always_clip: bool = False) -> dict:
    """The propagation loop (nlspnmodel.py:340-381) from prologued inputs: p0 (the
    blended [clamped] pred_init iteration 1 propagates), the blended confidence, the
    normalised (K+1)-tap affinity and the inserted 2(K+1)-plane offsets — what
    heads.head_epilogue_prologue writes (or propagate's own step 1).  Inference only.
    Returns {'pred', 'pred_inter' (T views), 'pred_inter_tensor'}."""
    kh, kw = kernel_geometry(kernel)
    K = kh * kw - 1
    for n, t in (("p0", p0), ("dep", dep), ("confidence", confidence), ("aff", aff), ("offset", offset)):
        _cuda(n, t)
    B, _, H, W = p0.shape
    dt = p0.dtype
    for n, t, c in (("p0", p0, 1), ("dep", dep, 1), ("confidence", confidence, 1), ("aff", aff, K + 1),
                    ("offset", offset, 2 * (K + 1))):
        if t is not None and (tuple(t.shape) != (B, c, H, W) or not t.is_contiguous() or t.dtype != dt):
            raise RuntimeError(f"{n} must be a contiguous {(B, c, H, W)} tensor of p0's dtype")
    if preserve_input and dep is None:
        raise RuntimeError("preserve_input requires dep")
    T = int(prop_time)
    kw_ = dict(dtype=dt, device=p0.device)
    pred_inter = torch.empty((T, B, 1, H, W), **kw_)
    pred = torch.empty((B, 1, H, W), **kw_)
    ws = torch.empty(_lib.get().nlspn_workspace_bytes(_dtype_code(p0), B, H, W) // 4, dtype=torch.int32,
                     device=p0.device)
    flags = (_lib.PRESERVE_INPUT if preserve_input else 0) | (_lib.ALWAYS_CLIP if always_clip else 0)
    with torch.cuda.device(p0.device):
        _lib.check_resident()
        _lib.check(_lib.get().nlspn_propagate_normalized(
            _dtype_code(p0), _ptr(p0), _ptr(dep), _ptr(confidence), _ptr(aff), _ptr(offset), _ptr(pred_inter),
            _ptr(pred), _ptr(ws), B, H, W, kh, kw, T, flags, _stream(p0.device)))
    return {"pred": pred, "pred_inter": list(pred_inter.unbind(0)), "pred_inter_tensor": pred_inter}


class PropagationPlan:
    """propagate() captured once (nlspn_plan_create) over fixed input/output buffers;
    replay() re-runs the whole section (the recorded launches re-issued directly, or
    one hipGraphLaunch).  Refill the input tensors in place between replays; γ is
    read on the device.  Resident launches of one device are serialised across
    streams by the library; check() raises if one aborted."""

    def __init__(self, pred_init, dep, confidence, aff, offset, gamma, *, prop_time=18, affinity="TGASS",
                 kernel=(3, 3), preserve_input=True, always_clip=False, return_offset=True):
        kh, kw = kernel_geometry(kernel)
        self.device = pred_init.device
        self.outputs = _alloc_outputs(pred_init, kh * kw - 1, prop_time, offset is not None and return_offset,
                                      confidence is not None)
        args, g = _propagate_args(pred_init, dep, confidence, aff, offset, gamma, kernel, prop_time, affinity,
                                  preserve_input, always_clip, self.outputs)
        self._keep = (pred_init, dep, confidence, aff, offset, g)  # buffers baked into the graph
        self._plan = ctypes.c_void_p()
        self._lib = _lib.get()
        with torch.cuda.device(self.device):
            _lib.check(self._lib.nlspn_plan_create(ctypes.byref(self._plan), *args))

    def replay(self) -> dict:
        with torch.cuda.device(self.device):
            _lib.check_resident()  # an earlier resident launch that aborted raises here
            _lib.check(self._lib.nlspn_plan_launch(self._plan, _stream(self.device)))
        o = self.outputs
        return {"pred": o["pred"], "pred_inter": list(o["pred_inter"].unbind(0)), "offset": o["offset"],
                "aff": o["aff"], "confidence": o["confidence"], "pred_inter_tensor": o["pred_inter"]}

    def check(self) -> None:
        """Wait for this device's queued work, then raise RuntimeError if a resident
        launch aborted (its outputs are NaN-filled; see nlspn_resident_status)."""
        torch.cuda.synchronize(self.device)
        _lib.check_resident(self.device)

    def close(self) -> None:
        if getattr(self, "_plan", None) is not None and self._plan.value:
            self._lib.nlspn_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# -------------------------------------------------------------- nn.Module
class NLSPNPropagation(nn.Module):
    """The propagation state and section of NLSPNModel (nlspnmodel.py:88-121, :317-383)
    as a module.  Reads the reference's args attribute names: prop_kernel (int, or an
    (kh, kw) tuple via args.prop_kernel_hw), affinity, affinity_gamma, prop_time,
    preserve_input, always_clip, conf_prop, offset.  Parameters keep the reference's
    state_dict names and shapes: aff_scale_const, w, b, w_conf."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        kernel = getattr(args, "prop_kernel_hw", None) or args.prop_kernel
        self.kh, self.kw = kernel_geometry(kernel)
        self.num_neighbors = self.kh * self.kw - 1
        self.ch_f = 1
        self.idx_ref = self.num_neighbors // 2
        if args.affinity == "TC":
            self.aff_scale_const = nn.Parameter(self.num_neighbors * torch.ones(1), requires_grad=False)
        elif args.affinity == "TGASS":
            self.aff_scale_const = nn.Parameter(args.affinity_gamma * self.num_neighbors * torch.ones(1))
        elif args.affinity in ("AS", "ASS"):
            self.aff_scale_const = nn.Parameter(torch.ones(1), requires_grad=False)
        else:
            raise NotImplementedError
        # dummy gathering parameters, kept so reference checkpoints load (nlspnmodel.py:107-114)
        self.w = nn.Parameter(torch.ones((self.ch_f, 1, self.kh, self.kw)), requires_grad=False)
        self.b = nn.Parameter(torch.zeros(self.ch_f), requires_grad=False)
        self.w_conf = nn.Parameter(torch.ones((1, 1, 1, 1)), requires_grad=False)

    def forward(self, pred_init, dep, off_aff, confidence=None) -> dict:
        a = self.args
        K = self.num_neighbors
        if a.offset:
            off, aff = off_aff[:, :2 * K], off_aff[:, 2 * K:]   # nlspnmodel.py:303-305
        else:
            off, aff = None, off_aff
        if not a.conf_prop:
            confidence = None
        out = propagate(pred_init, dep, confidence, aff, off, self.aff_scale_const, prop_time=a.prop_time,
                        affinity=a.affinity, kernel=(self.kh, self.kw), preserve_input=a.preserve_input,
                        always_clip=a.always_clip)
        return {"pred": out["pred"], "pred_init": pred_init, "pred_inter": out["pred_inter"],
                "offset": out["offset"], "aff": out["aff"], "gamma": self.aff_scale_const.data,
                "confidence": out["confidence"]}
