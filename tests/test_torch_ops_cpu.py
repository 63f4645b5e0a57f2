"""CPU: the torch operator layer (torch.ops.nlspn.*, csrc/nlspn_torch.cpp) loads, its
schemas mirror the reference's operator surface (vision.cpp:9-10 for the DCN pair),
and the fake kernels give torch.compile the right output shapes."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from nlspn_eccv20_amd import ops

pytestmark = pytest.mark.skipif(not ops.available(), reason="libnlspn_torch.so not built")

OPS = ("affinity_normalization", "prop_step", "propagate", "propagate_normalized", "modulated_deform_conv_forward",
       "modulated_deform_conv_backward")


def test_ops_registered_with_schemas():
    for name in OPS:
        schema = str(getattr(torch.ops.nlspn, name).default._schema)
        assert schema.startswith(f"nlspn::{name}("), schema
    fwd = str(torch.ops.nlspn.modulated_deform_conv_forward.default._schema)
    # DCN.modulated_deform_conv_forward's argument list (vision.cpp:9, modulated_deform_conv.h:10-23)
    for arg in ("input", "weight", "bias", "offset", "mask", "kernel_h", "kernel_w", "stride_h", "stride_w",
                "pad_h", "pad_w", "dilation_h", "dilation_w", "group", "deformable_group", "im2col_step"):
        assert f" {arg}" in fwd, arg


def test_fake_shapes():
    with FakeTensorMode():
        d = dict(device="cuda")
        x = torch.empty(2, 1, 8, 16, **d)
        raw = torch.empty(2, 24, 8, 16, **d)
        g = torch.empty(1, **d)
        pred, inter, aff, off, conf = torch.ops.nlspn.propagate(x, x, x, raw[:, 16:], raw[:, :16], g, 5)
        assert inter.shape == (5, 2, 1, 8, 16) and aff.shape == (2, 9, 8, 16) and off.shape == (2, 18, 8, 16)
        assert conf.shape == (2, 1, 8, 16) and pred.shape == (2, 1, 8, 16)
        pred, inter, aff, off, conf = torch.ops.nlspn.propagate(x, x, None, raw[:, 16:], None, g, 3)
        assert off is None and conf is None
        assert torch.ops.nlspn.affinity_normalization(raw[:, 16:], g, "TGASS").shape == (2, 9, 8, 16)
        assert torch.ops.nlspn.prop_step(x, x, x, aff, off, 3, 3).shape == x.shape
        pred, inter = torch.ops.nlspn.propagate_normalized(x, x, x, aff, off, 7)
        assert pred.shape == (2, 1, 8, 16) and inter.shape == (7, 2, 1, 8, 16)
        inp = torch.empty(2, 4, 13, 17, **d)
        w = torch.empty(6, 2, 3, 3, **d)
        o = torch.ops.nlspn.modulated_deform_conv_forward(inp, w, None, torch.empty(2, 36, 7, 9, **d),
                                                          torch.empty(2, 18, 7, 9, **d), 3, 3, 2, 2, 1, 1, 1, 1, 2,
                                                          2, 64)
        assert o.shape == (2, 6, 7, 9)


def test_ops_reject_cpu_tensors():
    """CPU tensors raise the reference's own error (modulated_deform_conv.h:43, :85):
    there is no CPU path behind the ops."""
    x = torch.zeros(1, 1, 4, 4)
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        torch.ops.nlspn.prop_step(x, None, None, torch.zeros(1, 9, 4, 4), None, 3, 3, False, False, False)
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        torch.ops.nlspn.propagate_normalized(x, x, x, torch.zeros(1, 9, 4, 4), torch.zeros(1, 18, 4, 4), 2)
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        torch.ops.nlspn.modulated_deform_conv_forward(x, torch.ones(1, 1, 3, 3), None, torch.zeros(1, 18, 4, 4),
                                                      torch.ones(1, 9, 4, 4), 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 64)
