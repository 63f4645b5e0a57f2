"""ORACLE (test infrastructure only) — numpy/ctypes front end of the C restatement.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  It loads ``oracle/build/liborc_nlspn.so`` (built by
``oracle/Makefile``), a plain-C restatement of the reference propagation section
(``src/model/nlspnmodel.py:179-381`` and the DCNv2 forward
``src/model/deformconv/src/cuda/modulated_deform_im2col_cuda.cuh:24-54,127-194``).
It is the checker, never the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborc_nlspn.so")

AFFINITY_KINDS = {"AS": 0, "ASS": 1, "TC": 2, "TGASS": 3}
PRESERVE = 1
ALWAYS_CLIP = 2

_lib = None


def build() -> str:
    """Compile the oracle with gcc (make)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        for sfx in ("f32", "f64"):
            getattr(_lib, f"orc_propagate_{sfx}").restype = ctypes.c_int
        _lib.orc_get_threads.restype = ctypes.c_int
    return _lib


def set_threads(n: int) -> None:
    lib().orc_set_threads(int(n))


def _sfx(dtype):
    dtype = np.dtype(dtype)
    if dtype == np.float32:
        return "f32", ctypes.c_float
    if dtype == np.float64:
        return "f64", ctypes.c_double
    raise TypeError(f"oracle supports float32/float64, got {dtype}")


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def affinity_normalization(aff_raw, kind="TGASS", gamma=4.0):
    """nlspnmodel.py:179-201 + :261-269 on a (B,K,H,W) array -> (B,K+1,H,W)."""
    dtype = aff_raw.dtype
    sfx, cr = _sfx(dtype)
    a = _c(aff_raw, dtype)
    B, K, H, W = a.shape
    out = np.empty((B, K + 1, H, W), dtype=dtype)
    getattr(lib(), f"orc_aff_norm_{sfx}")(
        _p(a), ctypes.c_longlong(K * H * W), B, K, ctypes.c_longlong(H * W),
        AFFINITY_KINDS[kind], cr(gamma), _p(out))
    return out


def off_insert(off_raw):
    """nlspnmodel.py:252-259 on a (B,2K,H,W) array -> (B,2(K+1),H,W)."""
    dtype = off_raw.dtype
    sfx, _ = _sfx(dtype)
    o = _c(off_raw, dtype)
    B, K2, H, W = o.shape
    K = K2 // 2
    out = np.empty((B, 2 * (K + 1), H, W), dtype=dtype)
    getattr(lib(), f"orc_off_insert_{sfx}")(
        _p(o), ctypes.c_longlong(K2 * H * W), B, K, ctypes.c_longlong(H * W), _p(out))
    return out


def mdcn_c1(im, off, mask, kh=3, kw=3, ph=None, pw=None):
    """DCNv2 forward for NLSPN's use (C=1, weight 1, bias 0); .cuh:127-194 + .cu:108-114."""
    dtype = im.dtype
    sfx, _ = _sfx(dtype)
    im, off, mask = (_c(x, dtype) for x in (im, off, mask))
    B, _, H, W = im.shape
    ph = (kh - 1) // 2 if ph is None else ph
    pw = (kw - 1) // 2 if pw is None else pw
    out = np.empty((B, 1, H, W), dtype=dtype)
    getattr(lib(), f"orc_mdcn_c1_{sfx}")(_p(im), _p(off), _p(mask), B, H, W, kh, kw, ph, pw, _p(out))
    return out


def prop_noffset(feat, aff):
    """nlspnmodel.py:209-224 (replicate-pad 3x3 gather)."""
    dtype = feat.dtype
    sfx, _ = _sfx(dtype)
    feat, aff = _c(feat, dtype), _c(aff, dtype)
    B, _, H, W = feat.shape
    out = np.empty((B, 1, H, W), dtype=dtype)
    getattr(lib(), f"orc_prop_noffset_{sfx}")(_p(feat), _p(aff), B, H, W, _p(out))
    return out


def propagate(pred_init, dep, conf, aff_raw, off_raw, gamma, *, kind="TGASS", kh=3, kw=3,
              prop_time=18, preserve_input=True, always_clip=False):
    """Whole propagation section, nlspnmodel.py:323-381.

    aff_raw (B,K,H,W) and off_raw (B,2K,H,W) or None (no-offset branch).
    Returns dict with pred, pred_inter (T,B,1,H,W), aff (B,K+1,H,W),
    offset (B,2(K+1),H,W) or None, confidence (B,1,H,W) or None.
    """
    dtype = pred_init.dtype
    sfx, cr = _sfx(dtype)
    pred_init, dep, conf, aff_raw, off_raw = (_c(x, dtype) for x in (pred_init, dep, conf, aff_raw, off_raw))
    B, _, H, W = pred_init.shape
    K = kh * kw - 1
    assert aff_raw.shape == (B, K, H, W), aff_raw.shape
    if off_raw is not None:
        assert off_raw.shape == (B, 2 * K, H, W), off_raw.shape
    flags = (PRESERVE if preserve_input else 0) | (ALWAYS_CLIP if always_clip else 0)
    pred_inter = np.empty((prop_time, B, 1, H, W), dtype=dtype)
    pred = np.empty((B, 1, H, W), dtype=dtype)
    aff_out = np.empty((B, K + 1, H, W), dtype=dtype)
    off_out = None if off_raw is None else np.empty((B, 2 * (K + 1), H, W), dtype=dtype)
    conf_out = None if conf is None else np.empty((B, 1, H, W), dtype=dtype)
    rc = getattr(lib(), f"orc_propagate_{sfx}")(
        _p(pred_init), _p(dep), _p(conf),
        _p(aff_raw), ctypes.c_longlong(K * H * W),
        _p(off_raw), ctypes.c_longlong(2 * K * H * W),
        cr(gamma), AFFINITY_KINDS[kind], kh, kw, prop_time, flags, B, H, W,
        _p(pred_inter), _p(pred), _p(aff_out), _p(off_out), _p(conf_out))
    if rc != 0:
        raise ValueError(f"oracle propagate rejected its arguments (code {rc})")
    return {"pred": pred, "pred_inter": pred_inter, "aff": aff_out,
            "offset": off_out, "confidence": conf_out}


def propagate_backward(pred_init, dep, conf, aff_raw, off_raw, gamma, grad_pred, grad_inter=None, *,
                       kind="TGASS", kh=3, kw=3, prop_time=18, preserve_input=True, always_clip=False):
    """Gradient of propagate() (autograd of nlspnmodel.py:323-381 through the DCN backward,
    modulated_deform_conv_cuda.cu:124-280).  Returns dict of grads: pred_init, confidence,
    aff (raw, B,K,H,W), offset (raw, B,2K,H,W) or None, gamma (float)."""
    dtype = pred_init.dtype
    sfx, cr = _sfx(dtype)
    pred_init, dep, conf, aff_raw, off_raw, grad_pred, grad_inter = (
        _c(x, dtype) for x in (pred_init, dep, conf, aff_raw, off_raw, grad_pred, grad_inter))
    B, _, H, W = pred_init.shape
    K = kh * kw - 1
    flags = (PRESERVE if preserve_input else 0) | (ALWAYS_CLIP if always_clip else 0)
    g_pi = np.empty((B, 1, H, W), dtype=dtype)
    g_conf = np.zeros((B, 1, H, W), dtype=dtype)
    g_aff = np.empty((B, K, H, W), dtype=dtype)
    g_off = None if off_raw is None else np.empty((B, 2 * K, H, W), dtype=dtype)
    g_gamma = np.zeros(1, dtype=dtype)
    fn = getattr(lib(), f"orc_propagate_backward_{sfx}")
    fn.restype = ctypes.c_int
    rc = fn(_p(pred_init), _p(dep), _p(conf), _p(aff_raw), ctypes.c_longlong(K * H * W),
            _p(off_raw), ctypes.c_longlong(2 * K * H * W), cr(gamma), AFFINITY_KINDS[kind], kh, kw, prop_time,
            flags, B, H, W, _p(grad_pred), _p(grad_inter), _p(g_pi), _p(g_conf), _p(g_aff), _p(g_off), _p(g_gamma))
    if rc != 0:
        raise ValueError(f"oracle backward rejected its arguments (code {rc})")
    return {"pred_init": g_pi, "confidence": g_conf if conf is not None else None, "aff": g_aff,
            "offset": g_off, "gamma": float(g_gamma[0])}


def _mdcn_shape(H, W, kh, kw, sh, sw, ph, pw, dh, dw):
    return (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1, (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1


def mdcn_forward(inp, weight, bias, offset, mask, stride=(1, 1), padding=(1, 1), dilation=(1, 1), group=1,
                 deformable_group=1):
    """Generic modulated DCNv2 forward (seam 2, vision.cpp:9): .cuh:127-194 + .cu:90-116."""
    dtype = inp.dtype
    sfx, _ = _sfx(dtype)
    inp, weight, offset, mask = (_c(x, dtype) for x in (inp, weight, offset, mask))
    bias = _c(bias, dtype)
    B, C, H, W = inp.shape
    Cout, _, kh, kw = weight.shape
    Ho, Wo = _mdcn_shape(H, W, kh, kw, *stride, *padding, *dilation)
    out = np.empty((B, Cout, Ho, Wo), dtype=dtype)
    getattr(lib(), f"orc_mdcn_fwd_{sfx}")(_p(inp), _p(weight), _p(bias), _p(offset), _p(mask), B, C, H, W, Cout, kh,
                                          kw, *stride, *padding, *dilation, group, deformable_group, _p(out))
    return out


def mdcn_backward(inp, weight, offset, mask, grad_output, stride=(1, 1), padding=(1, 1), dilation=(1, 1),
                  group=1, deformable_group=1, with_bias=True):
    """Generic modulated DCNv2 backward (seam 2, vision.cpp:10; .cu:124-280), including the
    reference's pad_w := pad_h in its col2im call (.cuh:371).  Returns
    (grad_input, grad_offset, grad_mask, grad_weight, grad_bias or None)."""
    dtype = inp.dtype
    sfx, _ = _sfx(dtype)
    inp, weight, offset, mask, grad_output = (_c(x, dtype) for x in (inp, weight, offset, mask, grad_output))
    B, C, H, W = inp.shape
    Cout, _, kh, kw = weight.shape
    gi, goff, gm, gw = (np.empty_like(x) for x in (inp, offset, mask, weight))
    gb = np.empty((Cout,), dtype=dtype) if with_bias else None
    rc = getattr(lib(), f"orc_mdcn_bwd_{sfx}")(
        _p(inp), _p(weight), _p(offset), _p(mask), _p(grad_output), B, C, H, W, Cout, kh, kw, *stride, *padding,
        *dilation, group, deformable_group, _p(gi), _p(goff), _p(gm), _p(gw), _p(gb))
    if rc != 0:
        raise MemoryError("oracle mdcn backward: allocation failed")
    return gi, goff, gm, gw, gb


def s2d_front(dep, w1, b1, w2, b2):
    """S2D pool pyramid + pool_convs + concat (src/model/nlspnmodel.py:437-459), numpy.

    dep (B, 1, H, W) sparse depth; w1 (8, 6[, 1, 1]), b1 (8), w2 (16, 8[, 1, 1]), b2 (16).
    Min pools s = 3, 5, 7, 9 (:441-447): -maxpool(where(dep == 0, -999, -dep)) with the
    pools' implicit -inf padding, then 999 -> 0; restated as the min over in-image cells
    of (dep != 0 ? dep : 999).  Max pools s = 11, 13 (:449-452).  pool_convs: two 1x1
    conv + ReLU (:455), accumulated in float64 and rounded once.  Returns
    (out (B, 17, H, W) = [pool_convs output, dep], pyramid (B, 6, H, W)), float32."""
    from numpy.lib.stride_tricks import sliding_window_view as swv

    d = np.asarray(dep, np.float32)[:, 0]
    B, H, W = d.shape
    pyr = np.empty((B, 6, H, W), np.float32)
    masked = np.where(d == 0, np.float32(999), d)
    for i, r in enumerate((1, 2, 3, 4)):
        p = np.pad(masked, ((0, 0), (r, r), (r, r)), constant_values=np.inf)
        m = swv(p, (2 * r + 1, 2 * r + 1), axis=(1, 2)).min(axis=(-1, -2))
        pyr[:, i] = np.where(m == 999, np.float32(0), m)
    for i, r in enumerate((5, 6)):
        p = np.pad(d, ((0, 0), (r, r), (r, r)), constant_values=-np.inf)
        pyr[:, 4 + i] = swv(p, (2 * r + 1, 2 * r + 1), axis=(1, 2)).max(axis=(-1, -2))
    w1 = np.asarray(w1, np.float64).reshape(8, 6)
    w2 = np.asarray(w2, np.float64).reshape(16, 8)
    h1 = np.maximum(np.einsum("oc,bchw->bohw", w1, pyr.astype(np.float64)) +
                    np.asarray(b1, np.float64).reshape(1, 8, 1, 1), 0).astype(np.float32)
    h2 = np.maximum(np.einsum("oc,bchw->bohw", w2, h1.astype(np.float64)) +
                    np.asarray(b2, np.float64).reshape(1, 16, 1, 1), 0).astype(np.float32)
    return np.concatenate([h2, d[:, None]], 1), pyr


def conv3x3(x, w, b):
    """3x3 / stride 1 / zero-pad 1 convolution with bias, float64 (nn.Conv2d as the
    reference's conv_bn_relu(..., bn=False) builds it, common.py:45-67): x (B, Ci, H, W),
    w (Co, Ci, 3, 3), b (Co) -> (B, Co, H, W)."""
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    B, Ci, H, W = x.shape
    p = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)))
    out = np.zeros((B, w.shape[0], H, W), np.float64)
    for dy in range(3):
        for dx in range(3):
            out += np.einsum("oc,bchw->bohw", w[:, :, dy, dx], p[:, :, dy:dy + H, dx:dx + W], optimize=True)
    return out + np.asarray(b, np.float64).reshape(1, -1, 1, 1)


def head_epilogue(fe1, off_aff_fd1, w_oa, b_oa, id_fd1=None, w_id=None, b_id=None, cf_fd1=None, w_cf=None,
                  b_cf=None):
    """The decoder's last three heads (src/model/nlspnmodel.py:296-315), float64:
    pred_init = ReLU(id_dec0(cat(id_fd1, fe1))) (:297), off_aff = off_aff_dec0(cat(
    off_aff_fd1, fe1)) (:301), confidence = Sigmoid(cf_dec0(cat(cf_fd1, fe1))) (:313).
    Returns (pred_init or None, off_aff, confidence or None) in float64."""
    cat = lambda fd: np.concatenate([np.asarray(fd, np.float64), np.asarray(fe1, np.float64)], 1)  # noqa: E731
    off_aff = conv3x3(cat(off_aff_fd1), w_oa, b_oa)
    pred_init = None if id_fd1 is None else np.maximum(conv3x3(cat(id_fd1), w_id, b_id), 0.0)
    conf = None if cf_fd1 is None else 1.0 / (1.0 + np.exp(-conv3x3(cat(cf_fd1), w_cf, b_cf)))
    return pred_init, off_aff, conf
