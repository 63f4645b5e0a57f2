"""Loader for the in-tree HIP library (``nlspn_eccv20_amd/lib/libnlspn_hip.so``).

The library exposes the C ABI declared in ``include/nlspn_prop.h``.  torch is
imported first on purpose: its bundled HIP runtime (soname ``libamdhip64.so.7``)
must be the one our library binds to, so that torch streams and device pointers
are valid in our calls.  There is no fallback: if the library is missing the
product path raises.
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch  # noqa: F401  (load torch's HIP runtime before our library)

_HERE = os.path.dirname(os.path.abspath(__file__))
# NLSPN_LIB_PATH: another build of the same ABI (A/B timing of library versions)
LIB_PATH = os.environ.get("NLSPN_LIB_PATH") or os.path.join(_HERE, "lib", "libnlspn_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "nlspn_prop.h")

DTYPE_F32, DTYPE_F16, DTYPE_F64 = 0, 1, 2  # F64: the seam-2 DCN entry points only
AFF_KINDS = {"AS": 0, "ASS": 1, "TC": 2, "TGASS": 3}
PRESERVE_INPUT, ALWAYS_CLIP = 0x1, 0x2
RESIDENT_FIRST = 0x100  # nlspn_time_propagate *resident: iteration 1 ran inside the resident launches
OFF_INSERTED, OFF_RAW = 0, 1
EINVAL, EUNSUPPORTED, EHIP, EABORTED = 1, 2, 3, 4

_vp, _i, _u, _i64, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_int64, ctypes.c_size_t
_fp = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes); mirrors include/nlspn_prop.h
SIGNATURES = {
    "nlspn_abi_version": (_i, []),
    "nlspn_last_error": (ctypes.c_char_p, []),
    "nlspn_affinity_normalize": (_i, [_i, _vp, _i64, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nlspn_s2d_pyramid": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp]),
    "nlspn_head_packed_size": (_i, [_i, _i, ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "nlspn_head_pack_weights": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    "nlspn_head_epilogue": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nlspn_head_epilogue_prologue": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _i, _i, _i, _i, _i, _i, _i, _u, _vp]),
    "nlspn_propagate_normalized": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _u, _vp]),
    "nlspn_prop_step": (_i, [_i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _i, _vp, _vp, _i, _i, _i, _i, _i, _u, _vp]),
    "nlspn_workspace_bytes": (_sz, [_i, _i, _i, _i]),
    "nlspn_propagate": (_i, [_i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                             _i, _i, _i, _i, _i, _i, _i, _u, _vp]),
    "nlspn_plan_create": (_i, [ctypes.POINTER(_vp), _i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _u]),
    "nlspn_plan_launch": (_i, [_vp, _vp]),
    "nlspn_plan_destroy": (_i, [_vp]),
    "nlspn_mdcn_forward": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                                _i, _i, _i, _i, _vp]),
    "nlspn_mdcn_backward": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i,
                                 _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nlspn_time_prop_step": (_i, [_i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _i, _vp, _i, _i, _i, _i, _i, _u, _i,
                                  _vp, _fp, _fp]),
    "nlspn_backward_workspace_bytes": (_sz, [_i, _i, _i, _i, _i]),
    "nlspn_propagate_backward": (_i, [_i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _vp, _i64, _vp, _i64, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _u, _vp]),
    "nlspn_prop_step_backward_workspace_bytes": (_sz, [_i, _i, _i]),
    "nlspn_prop_step_backward": (_i, [_i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _i, _i, _i, _i, _i, _u, _vp]),
    "nlspn_affinity_normalize_backward_workspace_bytes": (_sz, [_i, _i, _i, _i]),
    "nlspn_time_propagate": (_i, [_i, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _i, _i, _i, _i, _i, _i, _i, _u, _i, _vp, _vp, _vp, _vp]),
    "nlspn_resident_config": (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    "nlspn_resident_status": (_i, [_i]),
    "nlspn_affinity_normalize_backward": (_i, [_i, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nlspn_gconv_pack_layout": (_i, [_i, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "nlspn_gconv": (_i, [_i, _vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i,
                         ctypes.c_float, _i, _vp]),
    "nlspn_gconv_affnorm": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
}

# Entry points an A/B build (NLSPN_LIB_PATH) of an earlier round may lack; any other
# missing symbol fails the load (a stale or wrong library is refused up front)
AB_OPTIONAL = frozenset({"nlspn_resident_status", "nlspn_resident_config", "nlspn_gconv_pack_layout", "nlspn_gconv",
                         "nlspn_gconv_affnorm"})

_lib = None


class NlspnError(RuntimeError):
    """Raised when the HIP library rejects a call (mirrors the reference's c10::Error -> RuntimeError)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


def get() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"NLSPN HIP library not found at {LIB_PATH}; build it with "
                "`make -C nlspn_eccv20_amd/csrc` or __graft_entry__.build(). "
                "There is no CPU fallback for the propagation hot path.")
        lib = ctypes.CDLL(LIB_PATH)
        skipped = []
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(lib, name) and os.environ.get("NLSPN_LIB_PATH") and name in AB_OPTIONAL:
                skipped.append(name)  # A/B against an older build: entry points added since are absent
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if skipped:
            warnings.warn(f"NLSPN_LIB_PATH={LIB_PATH}: entry points absent from this build: {', '.join(skipped)}")
        _lib = lib
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        msg = get().nlspn_last_error().decode(errors="replace")
        raise NlspnError(rc, msg)


def check_resident(device=None) -> None:
    """Raise NlspnError (a RuntimeError) if a resident launch on `device` (default: the
    current one) aborted since the last check; clears the sticky word.  No device sync:
    an abort is seen once the aborted launch has finished."""
    lib = get()
    if not hasattr(lib, "nlspn_resident_status"):
        return
    if device is None:
        hit = lib.nlspn_resident_status(1)
    else:
        with torch.cuda.device(device):
            hit = lib.nlspn_resident_status(1)
    if hit:
        raise NlspnError(EABORTED, lib.nlspn_last_error().decode(errors="replace"))


def header_symbols() -> list[str]:
    """Function names declared in include/nlspn_prop.h (for export checks)."""
    import re

    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nlspn_[a-z0-9_]+)\s*\(", text)))
