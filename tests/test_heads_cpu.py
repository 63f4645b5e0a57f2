"""CPU: the head-epilogue oracle (oracle.head_epilogue, float64) is pinned to the
reference's own op sequence for the three heads (nlspnmodel.py:296-315: torch.cat,
nn.Conv2d(128, n, 3, padding=1), ReLU / Sigmoid), and the host wrapper rejects what
the kernel does not take."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import oracle as O


def _heads(C=16, nout=24, seed=0):
    torch.manual_seed(seed)
    mk = lambda n: nn.Conv2d(2 * C, n, 3, stride=1, padding=1).double()  # noqa: E731
    return mk(nout), mk(1), mk(1)


@pytest.mark.parametrize("nout,with_id,with_cf", [(24, True, True), (8, True, False), (48, False, True)])
def test_oracle_matches_reference_op_sequence(nout, with_id, with_cf):
    C = 16
    oa, idc, cfc = _heads(C, nout)
    g = torch.Generator().manual_seed(1)
    fe1, fd_oa, fd_id, fd_cf = (torch.rand((2, C, 11, 13), generator=g, dtype=torch.float64) for _ in range(4))
    with torch.no_grad():
        ref_oa = oa(torch.cat((fd_oa, fe1), 1))
        ref_id = torch.relu(idc(torch.cat((fd_id, fe1), 1)))
        ref_cf = torch.sigmoid(cfc(torch.cat((fd_cf, fe1), 1)))
    n = lambda t: t.detach().numpy()  # noqa: E731
    p, o, c = O.head_epilogue(n(fe1), n(fd_oa), n(oa.weight), n(oa.bias),
                              n(fd_id) if with_id else None, n(idc.weight), n(idc.bias),
                              n(fd_cf) if with_cf else None, n(cfc.weight), n(cfc.bias))
    assert np.abs(o - n(ref_oa)).max() < 1e-12
    if with_id:
        assert np.abs(p - n(ref_id)).max() < 1e-12
    else:
        assert p is None
    if with_cf:
        assert np.abs(c - n(ref_cf)).max() < 1e-12
    else:
        assert c is None


def test_head_epilogue_rejects_cpu_tensors():
    pytest.importorskip("nlspn_eccv20_amd.heads")
    from nlspn_eccv20_amd import _lib
    from nlspn_eccv20_amd.heads import head_epilogue
    try:
        _lib.get()
    except (ImportError, OSError):
        pytest.skip("HIP library not built")
    oa = nn.Conv2d(32, 24, 3, padding=1)
    x = torch.zeros((1, 16, 8, 8))
    with pytest.raises(RuntimeError, match="CUDA"):
        head_epilogue(x, x, oa)
    with pytest.raises(RuntimeError, match="both its decoder output"):
        head_epilogue(x, x, oa, id_fd1=x)


def test_fused_prologue_host_checks():
    """The fused-prologue entry points refuse what their kernels do not take (CPU
    tensors, a missing id head, a non-K=8 head) before any launch."""
    from nlspn_eccv20_amd import _lib, propagate_normalized
    from nlspn_eccv20_amd.heads import head_epilogue_prologue
    try:
        _lib.get()
    except (ImportError, OSError):
        pytest.skip("HIP library not built")
    x = torch.zeros((1, 1, 8, 8))
    with pytest.raises(RuntimeError, match="CUDA"):
        propagate_normalized(x, x, x, torch.zeros((1, 9, 8, 8)), torch.zeros((1, 18, 8, 8)), 3)
    oa = nn.Conv2d(32, 24, 3, padding=1)
    f = torch.zeros((1, 16, 8, 8))
    with pytest.raises(RuntimeError, match="id_fd1"):
        head_epilogue_prologue(f, f, oa, None, None, x, torch.ones(1))
    with pytest.raises(RuntimeError, match="K=8"):
        head_epilogue_prologue(f, f, nn.Conv2d(32, 48, 3, padding=1), f, nn.Conv2d(32, 1, 3, padding=1), x,
                               torch.ones(1))
