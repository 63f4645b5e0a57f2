"""CPU-side checks of the C ABI library and the host mirror (no GPU compute calls):
the library loads, exports every symbol include/nlspn_prop.h declares, and rejects
bad arguments with reference-style errors before touching the device."""
import ctypes
import subprocess
import types

import numpy as np
import pytest
import torch

from nlspn_eccv20_amd import _lib
from nlspn_eccv20_amd.propagation import NLSPNPropagation, kernel_geometry, off_insert, propagate


def test_library_exports_header_symbols():
    lib = _lib.get()
    declared = _lib.header_symbols()
    assert len(declared) >= 10
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if line.strip()}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == set(declared)  # ctypes bindings cover the whole header
    for s in declared:
        assert getattr(lib, s) is not None


def test_abi_version_and_workspace():
    lib = _lib.get()
    assert lib.nlspn_abi_version() == 3
    # resident kernel sync words (a 16-B multiple: one 128-B line per workgroup + the abort line)
    assert lib.nlspn_workspace_bytes(0, 8, 228, 304) == 513 * 128  # one 128-B sync line per resident part
    assert lib.nlspn_resident_config(0, 8, 228, 304, 3, 3, 18, 1, None, None, None) == 0  # no GPU here
    # backward: dL/df ping-pong, then (from a 128-B line) the resident pass 1's sync words (an
    # abort / registration line, one arrival line per part (up to 256) and an 8-word adjacency
    # row per part), K planes of G, dL/dconf' and room for two dL/dgamma partials per 8x32 tile
    B, H, W, K = 8, 228, 304, 8
    tiles = B * ((H + 7) // 8) * ((W + 31) // 32)
    N = B * H * W
    gf = (2 * N + 31) // 32 * 32  # the two dL/df planes, line-aligned: the sync words follow them
    assert lib.nlspn_backward_workspace_bytes(B, H, W, 3, 3) == 4 * (gf + 32 * 257 + 256 * 8 + N * (1 + K) + 2 * tiles)
    assert lib.nlspn_backward_workspace_bytes(0, H, W, 3, 3) == 0
    assert lib.nlspn_prop_step_backward_workspace_bytes(B, H, W) == 4 * 2 * B * H * W
    assert lib.nlspn_affinity_normalize_backward_workspace_bytes(B, K, H, W) > 0


def _call_step(**over):
    lib = _lib.get()
    p = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    a = dict(dtype=0, p_in=p, conf=None, dep=p, aff=p, aff_bs=9 * 4 * 4, off=p, off_bs=16 * 4 * 4, layout=1,
             p_out=p, pred_out=None, B=1, H=4, W=4, kh=3, kw=3, flags=1, stream=None)
    a.update(over)
    rc = lib.nlspn_prop_step(*a.values())
    return rc, lib.nlspn_last_error().decode()


@pytest.mark.parametrize("over,code,msg", [
    (dict(B=0), _lib.EINVAL, "empty input"),
    (dict(kh=2, kw=2), _lib.EINVAL, "only odd kernel"),
    (dict(dtype=7), _lib.EUNSUPPORTED, "dtype"),
    (dict(dep=None), _lib.EINVAL, "preserve_input requires dep"),
    (dict(aff_bs=8), _lib.EINVAL, "aff batch stride"),
    (dict(off_bs=3), _lib.EINVAL, "offset batch stride"),
    (dict(kh=9, kw=9, aff_bs=82 * 16, off_bs=160 * 16), _lib.EUNSUPPORTED, "no kernel instantiation"),
    (dict(off=None, kh=5, kw=5, aff_bs=25 * 16), _lib.EUNSUPPORTED, "no-offset propagation is 3x3"),
])
def test_step_validation(over, code, msg):
    rc, err = _call_step(**over)
    assert rc == code and msg in err, (rc, err)


def test_propagate_validation():
    lib = _lib.get()
    p = ctypes.c_void_p(16)
    rc = lib.nlspn_propagate(0, p, p, p, p, 8 * 16, p, 16 * 16, p, p, p, p, None, p, p,
                             1, 4, 4, 3, 3, 0, 3, 1, None)
    assert rc == _lib.EINVAL and "prop_time" in lib.nlspn_last_error().decode()
    rc = lib.nlspn_propagate(0, p, p, p, p, 8 * 16, p, 16 * 16, p, p, p, p, None, p, p,
                             1, 4, 4, 3, 3, 18, 9, 1, None)
    assert rc == _lib.EINVAL and "affinity kind" in lib.nlspn_last_error().decode()
    rc = lib.nlspn_mdcn_forward(0, p, p, None, p, p, p, 1, 3, 8, 8, 4, 3, 3, 1, 1, 1, 1, 1, 1, 2, 1, None)
    assert rc == _lib.EINVAL and "must divide group" in lib.nlspn_last_error().decode()
    rc = lib.nlspn_mdcn_backward(0, p, p, p, p, p, p, p, p, p, None, 1, 3, 8, 8, 4, 3, 3, 1, 1, 1, 1, 1, 1, 2, 1,
                                 None)
    assert rc == _lib.EINVAL and "must divide group" in lib.nlspn_last_error().decode()
    rc = lib.nlspn_mdcn_backward(1, p, p, p, p, p, p, p, p, p, None, 1, 4, 8, 8, 4, 3, 3, 1, 1, 1, 1, 1, 1, 2, 1,
                                 None)
    assert rc == _lib.EUNSUPPORTED and "float32" in lib.nlspn_last_error().decode()


def test_host_requires_cuda_tensors():
    x = torch.zeros(1, 1, 4, 4)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        propagate(x, x, x, torch.zeros(1, 8, 4, 4), torch.zeros(1, 16, 4, 4), torch.ones(1))


def test_kernel_geometry():
    assert kernel_geometry(3) == (3, 3)
    assert kernel_geometry((1, 17)) == (1, 17)
    with pytest.raises(AssertionError):
        kernel_geometry(4)


def test_off_insert_matches_oracle(oracle):
    off = np.random.default_rng(0).standard_normal((2, 16, 5, 7)).astype(np.float32)
    np.testing.assert_array_equal(off_insert(torch.from_numpy(off)).numpy(), oracle.off_insert(off))


def test_module_state_dict_keys_match_reference():
    args = types.SimpleNamespace(prop_kernel=3, affinity="TGASS", affinity_gamma=0.5, prop_time=18,
                                 preserve_input=True, always_clip=False, conf_prop=True, offset=True)
    m = NLSPNPropagation(args)
    sd = m.state_dict()
    assert set(sd) == {"aff_scale_const", "w", "b", "w_conf"}  # nlspnmodel.py:93-114
    assert sd["w"].shape == (1, 1, 3, 3) and float(sd["aff_scale_const"]) == 4.0
    assert m.aff_scale_const.requires_grad  # TGASS gamma is learnable (:97-99)
    args.affinity = "TC"
    assert float(NLSPNPropagation(args).aff_scale_const) == 8.0
