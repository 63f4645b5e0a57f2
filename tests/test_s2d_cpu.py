"""CPU: the S2D oracle restatement (oracle.s2d_front) pinned against the reference's
own torch ops (src/model/nlspnmodel.py:437-459: torch.where + nn.MaxPool2d + 1x1
conv/ReLU + cat), run here on CPU; and the library exports the S2D entry point."""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from nlspn_eccv20_amd import _lib
from oracle import oracle as O


def _torch_reference(dep, w1, b1, w2, b2):
    pyr = []
    for s in (3, 5, 7, 9):  # :441-447
        pool = nn.MaxPool2d(kernel_size=s, stride=1, padding=s // 2)
        z = -pool(torch.where(dep == 0, -999 * torch.ones_like(dep), -dep))
        pyr.append(torch.where(z == 999, torch.zeros_like(dep), z))
    for s in (11, 13):  # :449-452
        pyr.append(nn.MaxPool2d(kernel_size=s, stride=1, padding=s // 2)(dep))
    pyr = torch.cat(pyr, 1)
    h = F.relu(F.conv2d(F.relu(F.conv2d(pyr, w1, b1)), w2, b2))  # :455
    return torch.cat([h, dep], 1), pyr  # :459


def _case(B, H, W, density, seed):
    g = torch.Generator().manual_seed(seed)
    dep = torch.rand((B, 1, H, W), generator=g) * 10
    dep = torch.where(torch.rand((B, 1, H, W), generator=g) < density, dep, torch.zeros_like(dep))
    w1, b1 = torch.randn((8, 6, 1, 1), generator=g) * 0.5, torch.randn(8, generator=g) * 0.1
    w2, b2 = torch.randn((16, 8, 1, 1), generator=g) * 0.5, torch.randn(16, generator=g) * 0.1
    return dep, w1, b1, w2, b2


def test_oracle_matches_reference_ops():
    for B, H, W, density, seed in ((2, 40, 56, 0.05, 1), (1, 17, 23, 0.3, 2), (1, 9, 9, 0.0, 3), (1, 30, 30, 1.0, 4)):
        args = _case(B, H, W, density, seed)
        ref_out, ref_pyr = _torch_reference(*args)
        out, pyr = O.s2d_front(*(a.numpy() for a in args))
        assert np.array_equal(pyr, ref_pyr.numpy())  # pools: exact
        np.testing.assert_allclose(out, ref_out.numpy(), rtol=1e-5, atol=1e-5)
        assert np.array_equal(out[:, 16], args[0][:, 0].numpy())


def test_library_exports_s2d():
    assert hasattr(_lib.get(), "nlspn_s2d_pyramid")

