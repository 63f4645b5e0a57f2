"""GPU: the fused S2D front (nlspn_s2d_pyramid) against the oracle restatement
(oracle.s2d_front, pinned to the reference's torch ops in test_s2d_cpu.py) and its
weight gradients against torch autograd through the reference's ops.

Bar: the pool pyramid and the dep channel BIT-EXACT (min / max selections); the two
1x1 conv + ReLU layers within 1e-5 (MIOpen's and the oracle's summation orders
differ from the kernel's index order)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from nlspn_eccv20_amd import _lib
from nlspn_eccv20_amd.model import S2D
from nlspn_eccv20_amd.s2d import _run, s2d_front
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(B, H, W, density, seed):
    g = torch.Generator().manual_seed(seed)
    dep = torch.rand((B, 1, H, W), generator=g) * 80
    dep = torch.where(torch.rand((B, 1, H, W), generator=g) < density, dep, torch.zeros_like(dep))
    w1, b1 = torch.randn((8, 6, 1, 1), generator=g) * 0.3, torch.randn(8, generator=g) * 0.1
    w2, b2 = torch.randn((16, 8, 1, 1), generator=g) * 0.3, torch.randn(16, generator=g) * 0.1
    return dep, w1, b1, w2, b2


@pytest.mark.parametrize("B,H,W,density", [
    (8, 228, 304, 500 / (228 * 304)),   # NYU sampling density
    (4, 240, 1216, 0.05),               # KITTI-like
    (1, 5, 7, 0.5),                     # smaller than the 13x13 window
    (2, 33, 70, 0.0),                   # no depth at all: min pools 0
    (1, 20, 20, 1.0),                   # dense
])
def test_s2d_kernel_vs_oracle(B, H, W, density):
    args = _case(B, H, W, density, seed=B * H + W)
    ref_out, ref_pyr = O.s2d_front(*(a.numpy() for a in args))
    out, pyr = _run(*(a.to(DEV) for a in args), want_pyr=True)
    torch.cuda.synchronize()
    assert np.array_equal(pyr.cpu().numpy(), ref_pyr)
    o = out.cpu().numpy()
    assert np.array_equal(o[:, 16], ref_out[:, 16])
    np.testing.assert_allclose(o[:, :16], ref_out[:, :16], rtol=1e-5, atol=1e-5)


def test_s2d_weight_gradients_vs_torch():
    dep, w1, b1, w2, b2 = (a.to(DEV) for a in _case(2, 64, 96, 0.05, seed=9))
    params = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    out = s2d_front(dep, *params)
    g = torch.randn(out.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
    grads = torch.autograd.grad(out, params, g)
    _, pyr = O.s2d_front(*(a.cpu().numpy() for a in (dep, w1, b1, w2, b2)))
    rp = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    h = F.relu(F.conv2d(F.relu(F.conv2d(torch.from_numpy(pyr).to(DEV), rp[0], rp[1])), rp[2], rp[3]))
    ref = torch.autograd.grad(h, rp, g[:, :16])
    # both sides are MIOpen weight-gradient reductions over 12,288 pixels (its
    # algorithms may accumulate in different orders run to run): f32 reduction bar
    for a, r in zip(grads, ref):
        torch.testing.assert_close(a, r, rtol=1e-3, atol=1e-3)


def test_model_s2d_uses_kernel_and_matches_cpu_module():
    torch.manual_seed(3)
    m = S2D()
    dep = _case(2, 48, 64, 0.1, seed=5)[0]
    with torch.no_grad():
        ref = m(dep)                      # CPU tensors: the reference's torch ops
        out = m.to(DEV)(dep.to(DEV))      # GPU: the fused front + MIOpen 3x3 conv
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-4, atol=1e-4)


def test_s2d_rejects_bad_input():
    dep, w1, b1, w2, b2 = (a.to(DEV) for a in _case(1, 8, 8, 0.5, seed=1))
    with pytest.raises(RuntimeError):
        s2d_front(dep.double(), w1, b1, w2, b2)
    with pytest.raises(_lib.NlspnError):
        _lib.check(_lib.get().nlspn_s2d_pyramid(_lib.DTYPE_F16, None, None, None, None, None, None, None, 1, 1, 1,
                                                None))
