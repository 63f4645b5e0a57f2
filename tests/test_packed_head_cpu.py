"""CPU: host logic of the propagation autograd wrapper (no GPU calls)."""
import torch


def test_packed_head_detection():
    """propagation._packed_head: only the (B, 3K, H, W) head output sliced as the
    reference slices it (offsets first, nlspnmodel.py:304-305) is taken as packed."""
    from nlspn_eccv20_amd.propagation import _packed_head
    K = 8
    oa = torch.zeros((2, 3 * K, 6, 8), requires_grad=True)
    assert _packed_head(oa[:, 2 * K:], oa[:, :2 * K]) is oa
    assert _packed_head(oa[:, :K], oa[:, K:]) is None                       # other order
    assert _packed_head(oa[:, 2 * K:], None) is None                        # no-offset branch
    assert _packed_head(oa.detach()[:, 2 * K:], oa.detach()[:, :2 * K]) is None  # no grad wanted
    other = torch.zeros((2, 2 * K, 6, 8), requires_grad=True)
    assert _packed_head(oa[:, 2 * K:], other) is None                       # different tensors
    big = torch.zeros((2, 3 * K + 1, 6, 8), requires_grad=True)
    assert _packed_head(big[:, 2 * K:3 * K], big[:, :2 * K]) is None       # not exactly 3K planes


def test_packed_head_requires_grad_and_strides():
    """slices cut off from autograd, or with strides other than the base's,
    are not taken as packed (the gradient would reach a head output the caller cut
    off, or be written with the wrong layout)."""
    from nlspn_eccv20_amd.propagation import _packed_head
    K = 8
    oa = torch.zeros((2, 3 * K, 6, 8), requires_grad=True)
    with torch.no_grad():
        aff_ng, off_ng = oa[:, 2 * K:], oa[:, :2 * K]
    assert _packed_head(aff_ng, off_ng) is None                  # sliced under no_grad
    assert _packed_head(oa[:, 2 * K:], off_ng) is None
    odd = oa.as_strided((2, K, 6, 8), (3 * K * 48 - 48, 48, 8, 1), 2 * K * 48)
    assert _packed_head(odd, oa[:, :2 * K]) is None              # batch stride differs from the base
