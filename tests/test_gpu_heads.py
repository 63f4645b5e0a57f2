"""GPU: the head-epilogue kernel (nlspn_head_epilogue) against the float64 oracle of
the reference's three heads (nlspnmodel.py:296-315) and against torch's own f32
convolutions on the same device (what the reference runs).  f32 operands and
products, f32 accumulation in a different order: the bar is f32 rounding of a
1152-term sum — |got - ref64| <= 2e-6 * (sum_k |w_k x_k| + |b|), per element."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from nlspn_eccv20_amd.heads import HeadWeights, head_epilogue
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _case(B, C, H, W, nout, with_id=True, with_cf=True, seed=0, scale=1.0):
    torch.manual_seed(seed)
    oa = nn.Conv2d(2 * C, nout, 3, padding=1).to(DEV)
    idc = nn.Conv2d(2 * C, 1, 3, padding=1).to(DEV) if with_id else None
    cfc = nn.Conv2d(2 * C, 1, 3, padding=1).to(DEV) if with_cf else None
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    src = [torch.rand((B, C, H, W), device=DEV, generator=g) * scale for _ in range(4)]
    return oa, idc, cfc, src


def _bound(x_fd, fe1, w, b):
    """sum_k |w_k||x_k| + |b| per output element (float64), the scale of f32 rounding."""
    return O.conv3x3(np.abs(np.concatenate([x_fd, fe1], 1)), np.abs(w), np.abs(b))


def _check(got, ref, bound):
    err = np.abs(got.double().cpu().numpy() - ref)
    ratio = (err / (bound + 1e-30)).max()
    assert ratio <= 2e-6, f"max error / (sum |w x|) = {ratio:.3g}"
    return ratio


@pytest.mark.parametrize("B,C,H,W,nout,with_id,with_cf", [
    (2, 64, 40, 64, 24, True, True),      # K=8 with offsets (the default model), W % 4 == 0
    (2, 64, 37, 50, 24, True, True),      # partial tiles, W % 4 != 0 (scalar loads)
    (1, 64, 9, 8, 8, True, False),        # no offsets (nout = K), no confidence head
    (2, 32, 24, 96, 48, False, True),     # K=16 (1x17 geometry, 2 M-blocks), no id head
    (1, 64, 20, 36, 72, True, True),      # K=24 (5x5, 3 M-blocks)
    (1, 16, 13, 40, 144, True, True),     # K=48 (7x7, 5 M-blocks)
])
def test_head_epilogue_vs_oracle(B, C, H, W, nout, with_id, with_cf):
    oa, idc, cfc, (fe1, fd_oa, fd_id, fd_cf) = _case(B, C, H, W, nout, with_id, with_cf)
    with torch.no_grad():
        p, o, c = head_epilogue(fe1, fd_oa, oa, fd_id if with_id else None, idc, fd_cf if with_cf else None, cfc)
    torch.cuda.synchronize()
    n = lambda t: None if t is None else t.detach().double().cpu().numpy()  # noqa: E731
    rp, ro, rc = O.head_epilogue(n(fe1), n(fd_oa), n(oa.weight), n(oa.bias),
                                 n(fd_id) if with_id else None, n(idc.weight) if idc else None,
                                 n(idc.bias) if idc else None, n(fd_cf) if with_cf else None,
                                 n(cfc.weight) if cfc else None, n(cfc.bias) if cfc else None)
    _check(o, ro, _bound(n(fd_oa), n(fe1), n(oa.weight), n(oa.bias)))
    if with_id:
        _check(p, rp, _bound(n(fd_id), n(fe1), n(idc.weight), n(idc.bias)))
    else:
        assert p is None
    if with_cf:
        # sigmoid' <= 1/4: the pre-activation bound carries over
        _check(c, rc, _bound(n(fd_cf), n(fe1), n(cfc.weight), n(cfc.bias)))
    else:
        assert c is None


def test_head_epilogue_vs_torch_convs_nyu_size():
    """The reference's op sequence in f32 on the GPU (torch.cat + MIOpen conv) at the
    NYU size: same values up to f32 rounding."""
    oa, idc, cfc, (fe1, fd_oa, fd_id, fd_cf) = _case(2, 64, 228, 304, 24, seed=5)
    with torch.no_grad():
        p, o, c = head_epilogue(fe1, fd_oa, oa, fd_id, idc, fd_cf, cfc)
        ro = oa(torch.cat((fd_oa, fe1), 1))
        rp = torch.relu(idc(torch.cat((fd_id, fe1), 1)))
        rc = torch.sigmoid(cfc(torch.cat((fd_cf, fe1), 1)))
    for a, r in ((o, ro), (p, rp), (c, rc)):
        scale = r.abs().max().item() + 1.0
        assert (a - r).abs().max().item() <= 1e-5 * scale


def test_head_weights_cache_follows_updates():
    oa, idc, cfc, (fe1, fd_oa, fd_id, fd_cf) = _case(1, 16, 12, 32, 24)
    hw = HeadWeights()
    with torch.no_grad():
        _, o1, _ = head_epilogue(fe1, fd_oa, oa, weights=hw)
        oa.weight.mul_(2.0)   # in-place update: new version counter -> repacked
        oa.bias.mul_(2.0)
        _, o2, _ = head_epilogue(fe1, fd_oa, oa, weights=hw)
    assert torch.allclose(o2, 2 * o1, rtol=1e-5, atol=1e-5)


def test_head_epilogue_nonfinite_propagates():
    oa, idc, cfc, (fe1, fd_oa, fd_id, fd_cf) = _case(1, 16, 16, 32, 24)
    fe1[0, 3, 5, 7] = float("nan")
    with torch.no_grad():
        p, o, c = head_epilogue(fe1, fd_oa, oa, fd_id, idc, fd_cf, cfc)
    # the NaN reaches every output of the 3x3 neighbourhood of (5, 7) and nothing else
    bad = torch.isnan(o[0, 0])
    assert bad[4:7, 6:9].all() and bad.sum().item() == 9
    assert torch.isnan(p[0, 0, 5, 7]) and torch.isnan(c[0, 0, 5, 7])
