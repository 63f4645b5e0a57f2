"""Seam 1 of the drop-in: NLSPNModel with the reference's module tree and state_dict
keys, its encoder/decoder on stock PyTorch-ROCm (MIOpen convolutions) and its
propagation section on the MI355X kernels.

Mirrors XJTUXYC/NLSPN_ECCV20:
  src/model/nlspnmodel.py:23-159   NLSPNModel.__init__ (same attribute names / order)
  src/model/nlspnmodel.py:271-383  forward (encoder, heads, propagation, output dict)
  src/model/nlspnmodel.py:386-462  ConvGRU, S2D
  src/model/common.py:27-91        get_resnet18/34, conv_bn_relu, convt_bn_relu
The ResNet stages (`conv2..conv4` = torchvision resnet layer1..layer3) are built
here with torchvision's module naming (conv1/bn1/relu/conv2/bn2/downsample), since
torchvision is not part of this stack; reference checkpoints load unchanged.

Propagation: without the ConvGRU the whole section is one fused, differentiable
op (propagate: prop_time launches).  With use_GRU (the reference's forced default,
src/config.py:225-228) the affinity is re-estimated after every iteration
(nlspnmodel.py:365-373), so each iteration is prop_step + affinity_normalization
around the GRU's MIOpen convolutions; both are differentiable (step-level backward
kernels), so that mode trains too.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .propagation import (affinity_normalization, kernel_geometry, off_insert, prop_step, propagate,
                          propagate_normalized)
from .gru import GruConvs
from .heads import HeadWeights, head_epilogue, head_epilogue_prologue
from .s2d import s2d_front

__all__ = ["NLSPNModel", "ConvGRU", "S2D", "conv_bn_relu", "convt_bn_relu", "get_resnet18", "get_resnet34", "get",
           "SectionGraph"]

model_path = {"resnet18": "pretrained/resnet18.pth", "resnet34": "pretrained/resnet34.pth"}


# ---------------------------------------------------------------- common.py
def conv_bn_relu(ch_in, ch_out, kernel, stride=1, bn=True, relu=True, zero_init=False):
    """common.py:44-67: Sequential(conv[, bn][, relu])."""
    assert (kernel % 2) == 1, "only odd kernel is supported but kernel = {}".format(kernel)
    layers = [nn.Conv2d(ch_in, ch_out, kernel, stride, (kernel - 1) // 2, bias=not bn)]
    if zero_init:
        layers[0].weight.data.zero_()
        if not bn:
            layers[0].bias.data.zero_()
    if bn:
        layers.append(nn.BatchNorm2d(ch_out))
    if relu:
        layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


def convt_bn_relu(ch_in, ch_out, kernel, stride=1, padding=0, output_padding=0, bn=True, relu=True,
                  zero_init=False):
    """common.py:70-91: Sequential(convT[, bn][, relu])."""
    assert (kernel % 2) == 1, "only odd kernel is supported but kernel = {}".format(kernel)
    layers = [nn.ConvTranspose2d(ch_in, ch_out, kernel, stride, padding, output_padding, bias=not bn)]
    if zero_init:
        layers[0].weight.data.zero_()
        if not bn:
            layers[0].bias.data.zero_()
    if bn:
        layers.append(nn.BatchNorm2d(ch_out))
    if relu:
        layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


class BasicBlock(nn.Module):
    """ResNet basic block with torchvision's parameter names."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class _ResNetStages(nn.Module):
    """layer1..layer3 of a torchvision-style ResNet (the stages NLSPN keeps, nlspnmodel.py:45-52)."""

    def __init__(self, blocks):
        super().__init__()
        self.inplanes = 64
        self.layer1 = self._make(64, blocks[0], 1)
        self.layer2 = self._make(128, blocks[1], 2)
        self.layer3 = self._make(256, blocks[2], 2)
        for m in self.modules():  # torchvision's initialisation
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make(self, planes, n, stride):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, down)]
        self.inplanes = planes
        layers += [BasicBlock(planes, planes) for _ in range(1, n)]
        return nn.Sequential(*layers)


def _get_resnet(name, blocks, pretrained):
    net = _ResNetStages(blocks)
    if pretrained:  # common.py:27-42: torchvision resnet state_dict from pretrained/<name>.pth
        sd = torch.load(model_path[name], map_location="cpu", weights_only=True)
        net.load_state_dict({k: v for k, v in sd.items() if k.split(".")[0] in ("layer1", "layer2", "layer3")})
    return net


def get_resnet18(pretrained=True):
    return _get_resnet("resnet18", (2, 2, 2), pretrained)


def get_resnet34(pretrained=True):
    return _get_resnet("resnet34", (3, 4, 6), pretrained)


# ---------------------------------------------------------------- nlspnmodel.py
class ConvGRU(nn.Module):
    """nlspnmodel.py:386-403."""

    def __init__(self, args):
        super().__init__()
        c = args.GRU_hidden_dim + args.GRU_input_dim
        self.convz = nn.Conv2d(c, args.GRU_hidden_dim, 3, padding=1)
        self.convr = nn.Conv2d(c, args.GRU_hidden_dim, 3, padding=1)
        self.convq = nn.Conv2d(c, args.GRU_hidden_dim, 3, padding=1)

    def forward(self, h, x):
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(self.convz(hx))
        r = torch.sigmoid(self.convr(hx))
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=1)))
        return (1 - z) * h + z * q


class S2D(nn.Module):
    """nlspnmodel.py:406-462 (min/max-pool pyramid sparse-depth encoder)."""

    def __init__(self):
        super().__init__()
        self.min_pool_sizes = [3, 5, 7, 9]
        self.max_pool_sizes = [11, 13]
        # plain lists, as in the reference: the pools carry no parameters or state_dict keys
        self.min_pools = [nn.MaxPool2d(kernel_size=s, stride=1, padding=s // 2) for s in self.min_pool_sizes]
        self.max_pools = [nn.MaxPool2d(kernel_size=s, stride=1, padding=s // 2) for s in self.max_pool_sizes]
        in_channels = len(self.min_pool_sizes) + len(self.max_pool_sizes)
        self.pool_convs = nn.Sequential(conv_bn_relu(in_channels, 8, kernel=1, stride=1, bn=False),
                                        conv_bn_relu(8, 16, kernel=1, stride=1, bn=False))
        self.conv = conv_bn_relu(16 + 1, 32, kernel=3, stride=1, bn=False)

    def forward(self, dep):
        if dep.is_cuda and dep.dtype == torch.float32:  # the fused HIP front (s2d.py)
            c0, c1 = self.pool_convs[0][0], self.pool_convs[1][0]
            return self.conv(s2d_front(dep, c0.weight, c0.bias, c1.weight, c1.bias))
        pyr = []  # CPU tensors (host-side model tests): the reference's torch ops
        for pool in self.min_pools:
            z = -pool(torch.where(dep == 0, -999 * torch.ones_like(dep), -dep))
            pyr.append(torch.where(z == 999, torch.zeros_like(dep), z))
        for pool in self.max_pools:
            pyr.append(pool(dep))
        feat = self.pool_convs(torch.cat(pyr, dim=1))
        return self.conv(torch.cat([feat, dep], dim=1))


class NLSPNModel(nn.Module):
    """Drop-in for src/model/nlspnmodel.py:23-383 (same constructor argument, same
    submodule names, same forward(sample) -> dict)."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        kernel = getattr(args, "prop_kernel_hw", None) or args.prop_kernel
        self.kh, self.kw = kernel_geometry(kernel)
        self.num_neighbors = self.kh * self.kw - 1

        self.conv1_rgb = conv_bn_relu(3, 32, kernel=3, stride=1, bn=False)
        self.conv1_dep = conv_bn_relu(1, 32, kernel=3, stride=1, bn=False)
        if args.network == "resnet18":
            net = get_resnet18(not args.from_scratch)
        elif args.network == "resnet34":
            net = get_resnet34(not args.from_scratch)
        else:
            raise NotImplementedError
        self.conv2, self.conv3, self.conv4 = net.layer1, net.layer2, net.layer3
        del net
        self.conv5 = conv_bn_relu(256, 256, kernel=3, stride=2)
        self.dec4 = convt_bn_relu(256, 128, kernel=3, stride=2, padding=1, output_padding=1)
        self.dec3 = convt_bn_relu(128 + 256, 64, kernel=3, stride=2, padding=1, output_padding=1)
        self.dec2 = convt_bn_relu(64 + 128, 64, kernel=3, stride=2, padding=1, output_padding=1)
        self.id_dec1 = conv_bn_relu(64 + 64, 64, kernel=3, stride=1)
        self.id_dec0 = conv_bn_relu(64 + 64, 1, kernel=3, stride=1, bn=False, relu=True)
        self.off_aff_dec1 = conv_bn_relu(64 + 64, 64, kernel=3, stride=1)
        nout = 3 * self.num_neighbors if args.offset else self.num_neighbors
        self.off_aff_dec0 = conv_bn_relu(64 + 64, nout, kernel=3, stride=1, bn=False, relu=False,
                                         zero_init=args.zero_init_aff)
        if args.conf_prop:
            self.cf_dec1 = conv_bn_relu(64 + 64, 64, kernel=3, stride=1)
            self.cf_dec0 = nn.Sequential(nn.Conv2d(64 + 64, 1, kernel_size=3, stride=1, padding=1), nn.Sigmoid())
        self.ch_f = 1
        self.idx_ref = self.num_neighbors // 2
        if args.affinity in ("AS", "ASS", "TC", "TGASS"):
            if args.affinity == "TC":
                self.aff_scale_const = nn.Parameter(self.num_neighbors * torch.ones(1), requires_grad=False)
            elif args.affinity == "TGASS":
                self.aff_scale_const = nn.Parameter(args.affinity_gamma * self.num_neighbors * torch.ones(1))
            else:
                self.aff_scale_const = nn.Parameter(torch.ones(1), requires_grad=False)
        else:
            raise NotImplementedError
        self.w = nn.Parameter(torch.ones((self.ch_f, 1, self.kh, self.kw)), requires_grad=False)
        self.b = nn.Parameter(torch.zeros(self.ch_f), requires_grad=False)
        self.w_conf = nn.Parameter(torch.ones((1, 1, 1, 1)), requires_grad=False)
        self.stride, self.padding, self.dilation = 1, (self.kh - 1) // 2, 1
        self.groups, self.deformable_groups, self.im2col_step = self.ch_f, 1, 64
        if args.use_GRU:
            self.GRU = ConvGRU(args)
            self.encode_aff = nn.Sequential(
                conv_bn_relu(self.num_neighbors + 1, 16, kernel=3, stride=2, bn=False),
                conv_bn_relu(16, 2 * args.GRU_hidden_dim, kernel=3, stride=2, bn=False),
                conv_bn_relu(2 * args.GRU_hidden_dim, args.GRU_hidden_dim, kernel=3, stride=2, bn=False, relu=False),
                nn.Tanh())
            self.encode_dep = nn.Sequential(
                conv_bn_relu(1, 16, kernel=3, stride=2, bn=False),
                conv_bn_relu(16, 2 * args.GRU_input_dim, kernel=3, stride=2, bn=False),
                conv_bn_relu(2 * args.GRU_input_dim, args.GRU_input_dim, kernel=3, stride=2, bn=False))
            self.decode_aff = nn.Sequential(
                convt_bn_relu(args.GRU_hidden_dim, 2 * args.GRU_hidden_dim, kernel=3, stride=2, padding=1,
                              output_padding=1, bn=False),
                convt_bn_relu(2 * args.GRU_hidden_dim, 16, kernel=3, stride=2, padding=1, output_padding=1,
                              bn=False),
                convt_bn_relu(16, self.num_neighbors, kernel=3, stride=2, padding=1, output_padding=1, bn=False,
                              relu=False, zero_init=args.zero_init_aff))
        if args.use_S2D:
            self.S2D = S2D()
        self._head_weights = HeadWeights()  # packed head-epilogue weights (a cache, not state)
        # GRU mode at inference: encode_dep / encode_aff / ConvGRU / decode_aff as HIP
        # convolutions (gru.py); False keeps the torch modules (A/B, tests)
        self.native_gru = True
        self._gru_convs = GruConvs()
        params = nn.ParameterList([p for p in self.parameters() if p.requires_grad])
        self.param_groups = [{"params": params, "lr": args.lr}]

    def gru_channels_last(self):
        """Put the GRU-mode convolutions (ConvGRU, encode_aff / encode_dep, decode_aff) in
        channels_last: MIOpen's implicit-GEMM convolutions run NHWC, so this drops the
        NCHW<->NHWC transposes around every one of them.  With MIOpen's algorithm search
        (torch.backends.cudnn.benchmark) the GRU section at NYU B=8 goes 16.3 -> 11.2 ms
        (tools/gru_prof.py).  Numerics: the same convolutions in another layout."""
        if self.args.use_GRU:
            for sub in (self.GRU, self.encode_aff, self.encode_dep, self.decode_aff):
                sub.to(memory_format=torch.channels_last)
        return self

    @staticmethod
    def _crop(fd, fe):
        """The decoder-padding crop of nlspnmodel.py:161-174."""
        _, _, Hd, Wd = fd.shape
        _, _, He, We = fe.shape
        if Hd > He:
            fd = fd[:, :, :He, :]
        if Wd > We:
            fd = fd[:, :, :, :We]
        return fd

    @classmethod
    def _concat(cls, fd, fe, dim=1):
        """nlspnmodel.py:161-177: crop decoder padding, then concatenate."""
        return torch.cat((cls._crop(fd, fe), fe), dim=dim)

    def _decoder(self, sample):
        """Encoder + shared decoder + the heads' first layers, nlspnmodel.py:272-312:
        (fe1, id_fd1, off_aff_fd1, cf_fd1 or None), the decoder outputs cropped to fe1."""
        rgb, dep = sample["rgb"], sample["dep"]
        fe1_rgb = self.conv1_rgb(rgb)
        fe1_dep = self.S2D(dep) if self.args.use_S2D else self.conv1_dep(dep)
        fe1 = torch.cat((fe1_rgb, fe1_dep), dim=1)
        fe2 = self.conv2(fe1)
        fe3 = self.conv3(fe2)
        fe4 = self.conv4(fe3)
        fe5 = self.conv5(fe4)
        fd4 = self.dec4(fe5)
        fd3 = self.dec3(self._concat(fd4, fe4))
        fd2 = self.dec2(self._concat(fd3, fe3))
        id_fd1 = self.id_dec1(self._concat(fd2, fe2))
        off_aff_fd1 = self.off_aff_dec1(self._concat(fd2, fe2))
        cf_fd1 = self.cf_dec1(self._concat(fd2, fe2)) if self.args.conf_prop else None
        crop = lambda fd: None if fd is None else self._crop(fd, fe1)  # noqa: E731
        return fe1, crop(id_fd1), crop(off_aff_fd1), crop(cf_fd1)

    def _head_cache(self):
        """The packed head-weight cache, or None (pack per call) in a DataParallel replica:
        replicas share this module's __dict__ (so the cache) while their parameters are
        fresh broadcast copies whose storage and version counter can repeat across forwards
        with different master weights (src/main.py:366 runs the model under DataParallel)."""
        return None if getattr(self, "_is_replica", False) else self._head_weights

    def _fused_inference(self, fe1) -> bool:
        return fe1.is_cuda and not torch.is_grad_enabled() and fe1.dtype == torch.float32

    def heads(self, sample):
        """Encoder + decoder heads, nlspnmodel.py:272-315: (pred_init, off_aff, confidence)."""
        fe1, id_fd1, off_aff_fd1, cf_fd1 = self._decoder(sample)
        if self._fused_inference(fe1):
            # inference: the three last convolutions + bias/activation as one HIP kernel
            # reading fe1 and the decoder outputs in place (heads.py, nlspn_heads.h)
            return head_epilogue(fe1, off_aff_fd1, self.off_aff_dec0, id_fd1, self.id_dec0, cf_fd1,
                                 self.cf_dec0 if self.args.conf_prop else None, weights=self._head_cache())
        pred_init = self.id_dec0(torch.cat((id_fd1, fe1), 1))
        off_aff = self.off_aff_dec0(torch.cat((off_aff_fd1, fe1), 1))
        confidence = None
        if self.args.conf_prop:
            confidence = self.cf_dec0(torch.cat((cf_fd1, fe1), 1))
        return pred_init, off_aff, confidence

    def _aff_head(self, aff_feat):
        """nlspnmodel.py:228-234 (+ the _clip_as crop :237-250)."""
        if self._native_gru(aff_feat):
            gc = self._gru_convs
            # (K = 8: the last transposed conv normalises in its epilogue, nlspn_gconv_affnorm)
            aff = gc.decode_aff(gc.pack(self), aff_feat, (self.args.patch_height, self.args.patch_width),
                                gamma=self.aff_scale_const, kind=self.args.affinity)
            if aff.shape[1] == self.num_neighbors + 1:
                return aff
            return affinity_normalization(aff, self.aff_scale_const, self.args.affinity)
        aff = self.decode_aff(aff_feat)
        aff = aff[:, :, :self.args.patch_height, :self.args.patch_width].contiguous()
        return affinity_normalization(aff, self.aff_scale_const, self.args.affinity)

    def forward(self, sample):
        a = self.args
        if (not a.use_GRU and a.offset and (self.kh, self.kw) == (3, 3) and a.affinity in ("AS", "ASS", "TC", "TGASS")
                and torch.cuda.is_available() and sample["dep"].is_cuda and not torch.is_grad_enabled()):
            fe1, id_fd1, off_aff_fd1, cf_fd1 = self._decoder(sample)
            if self._fused_inference(fe1):
                return self._forward_fused(fe1, id_fd1, off_aff_fd1, cf_fd1, sample["dep"])
            return self.propagate_heads(*self._heads_from(fe1, id_fd1, off_aff_fd1, cf_fd1), sample["dep"])
        pred_init, off_aff, confidence = self.heads(sample)
        return self.propagate_heads(pred_init, off_aff, confidence, sample["dep"])

    def _heads_from(self, fe1, id_fd1, off_aff_fd1, cf_fd1):
        pred_init = self.id_dec0(torch.cat((id_fd1, fe1), 1))
        off_aff = self.off_aff_dec0(torch.cat((off_aff_fd1, fe1), 1))
        confidence = self.cf_dec0(torch.cat((cf_fd1, fe1), 1)) if self.args.conf_prop else None
        return pred_init, off_aff, confidence

    def _forward_fused(self, fe1, id_fd1, off_aff_fd1, cf_fd1, dep):
        """Inference, 3x3 / K=8 / offsets (the reference's NYU and KITTI models): the head
        convolutions with the propagation prologue fused into their epilogue
        (heads.head_epilogue_prologue: _off_insert, the affinity normalisation, the
        confidence / input blend, :296-348), then the loop from the prologued planes
        (propagation.propagate_normalized, :340-381).  The same output dict as
        propagate_heads, bit for bit given the same convolution sums."""
        a = self.args
        dep = dep.contiguous().float()  # as head_epilogue_prologue coerces it; propagate_normalized takes the same
        h = head_epilogue_prologue(fe1, off_aff_fd1, self.off_aff_dec0, id_fd1, self.id_dec0, dep,
                                   self.aff_scale_const, a.affinity, cf_fd1,
                                   self.cf_dec0 if a.conf_prop else None, a.preserve_input, a.always_clip,
                                   weights=self._head_cache())
        o = propagate_normalized(h["p0"], dep if a.preserve_input else None, h["confidence"], h["aff"],
                                 h["offset"], a.prop_time, (3, 3), a.preserve_input, a.always_clip)
        return {"pred": o["pred"], "pred_init": h["pred_init"], "pred_inter": o["pred_inter"],
                "offset": h["offset"], "aff": h["aff"], "gamma": self.aff_scale_const.data,
                "confidence": h["confidence"]}

    def propagate_heads(self, pred_init, off_aff, confidence, dep):
        """The propagation section, nlspnmodel.py:303-383, on the heads' outputs."""
        a = self.args
        assert self.ch_f == pred_init.shape[1]
        K = self.num_neighbors
        off = off_aff[:, :2 * K] if a.offset else None
        aff = off_aff[:, 2 * K:] if a.offset else off_aff
        if not a.use_GRU:
            o = propagate(pred_init, dep if a.preserve_input else None, confidence if a.conf_prop else None, aff,
                          off, self.aff_scale_const, prop_time=a.prop_time, affinity=a.affinity,
                          kernel=(self.kh, self.kw), preserve_input=a.preserve_input, always_clip=a.always_clip)
            return {"pred": o["pred"], "pred_init": pred_init, "pred_inter": o["pred_inter"], "offset": o["offset"],
                    "aff": o["aff"], "gamma": self.aff_scale_const.data, "confidence": o["confidence"]}
        return self._forward_gru(pred_init, dep, off, aff, confidence)

    def _forward_gru(self, pred_init, dep, off, aff_raw, confidence):
        """nlspnmodel.py:323-383 with use_GRU: the affinity is re-estimated after every
        iteration (:365-373).  Inference: iteration 1 runs the fused first step (prologue
        inside), later iterations prop_step on the GRU's freshly normalised affinity.
        With gradients: the prologue in torch, then T differentiable prop_steps
        (nlspn_prop_step_backward) and differentiable normalisations."""
        a = self.args
        if torch.is_grad_enabled():
            return self._forward_gru_train(pred_init, dep, off, aff_raw, confidence)
        o = propagate(pred_init, dep if a.preserve_input else None, confidence if a.conf_prop else None,
                      aff_raw, off, self.aff_scale_const, prop_time=1, affinity=a.affinity,
                      kernel=(self.kh, self.kw), preserve_input=a.preserve_input, always_clip=a.always_clip)
        new_pred = o["pred_inter"][0]
        aff, conf_eff = o["aff"], o["confidence"]
        list_pred = [new_pred]
        aff_feat = None
        for k in range(2, a.prop_time + 1):
            aff_feat = self._gru_update(aff_feat, aff, new_pred, k)
            aff = self._aff_head(aff_feat)
            new_pred = prop_step(new_pred, conf_eff, dep if a.preserve_input else None, aff, off,
                                 kernel=(self.kh, self.kw), offset_layout="raw", preserve_input=a.preserve_input,
                                 always_clip=a.always_clip)
            list_pred.append(new_pred)
        pred = new_pred if a.always_clip else torch.clamp(new_pred, min=0)
        return {"pred": pred, "pred_init": pred_init, "pred_inter": list_pred, "offset": o["offset"], "aff": aff,
                "gamma": self.aff_scale_const.data, "confidence": conf_eff}

    def _native_gru(self, x):
        """The GRU-mode convolutions run on the HIP kernels (gru.py): inference on CUDA with the
        reference's GRU architecture; training keeps the torch modules (their autograd)."""
        return (self.native_gru and x.is_cuda and not torch.is_grad_enabled() and x.dtype == torch.float32
                and GruConvs.supported(self))

    def _gru_update(self, aff_feat, aff, new_pred, k):
        """nlspnmodel.py:365-371: encode the new depth, (at the first update) encode the
        affinity, one ConvGRU step."""
        if self._native_gru(new_pred):
            gc = self._gru_convs
            P = gc.pack(self)
            dep_feat = gc.encode_dep(P, new_pred, self.args.max_depth)
            if k == 2:
                aff_feat = gc.encode_aff(P, aff)
            return gc.gru(P, aff_feat, dep_feat)
        dep_feat = self.encode_dep(new_pred / self.args.max_depth)
        if k == 2:
            aff_feat = self.encode_aff(aff)
        return self.GRU(h=aff_feat, x=dep_feat)

    def _forward_gru_train(self, pred_init, dep, off, aff_raw, confidence):
        a = self.args
        kern = (self.kh, self.kw)
        aff = affinity_normalization(aff_raw, self.aff_scale_const, a.affinity)
        conf_eff = confidence if a.conf_prop else None
        new_pred = pred_init
        if a.preserve_input:  # :328-334, :341-345
            mask_fix = (dep > 0.0).to(dep.dtype)
            if conf_eff is not None:
                conf_eff = (1.0 - mask_fix) * conf_eff + mask_fix
            new_pred = (1.0 - mask_fix) * new_pred + mask_fix * dep
        if a.always_clip:
            new_pred = torch.clamp(new_pred, min=0)
        new_pred = new_pred.contiguous()
        conf_eff = None if conf_eff is None else conf_eff.contiguous()
        list_pred = []
        aff_feat = None
        for k in range(1, a.prop_time + 1):
            if k > 1:
                aff_feat = self._gru_update(aff_feat, aff, new_pred, k)
                aff = self._aff_head(aff_feat)
            new_pred = prop_step(new_pred, conf_eff, dep if a.preserve_input else None, aff, off, kernel=kern,
                                 offset_layout="raw", preserve_input=a.preserve_input, always_clip=a.always_clip)
            list_pred.append(new_pred)
        pred = new_pred if a.always_clip else torch.clamp(new_pred, min=0)
        offset = off_insert(off) if off is not None else None
        return {"pred": pred, "pred_init": pred_init, "pred_inter": list_pred, "offset": offset, "aff": aff,
                "gamma": self.aff_scale_const.data, "confidence": conf_eff}


class SectionGraph:
    """NLSPNModel's propagation section (nlspnmodel.py:303-383) on fixed head-output
    buffers, captured once into one hipGraph (torch.cuda.CUDAGraph) and replayed with
    one launch: in GRU mode (the reference's forced default, src/config.py:225-228)
    the graph holds every iteration's MIOpen GRU convolutions, affinity
    normalisation and prop_step kernel (T-1 of each), so the per-iteration host
    launches disappear.  Inference only (no autograd through a replay).

    replay(pred_init, off_aff, confidence, dep) copies new head outputs into the
    captured buffers (any argument may be None to keep the previous values) and
    returns the output dict; its tensors are the graph's buffers, overwritten by
    the next replay."""

    def __init__(self, model, pred_init, off_aff, confidence, dep, warmup=2):
        self.model = model
        self.inputs = [None if t is None else t.detach().clone() for t in (pred_init, off_aff, confidence, dep)]
        side = torch.cuda.Stream(device=pred_init.device)
        side.wait_stream(torch.cuda.current_stream(pred_init.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(warmup):  # MIOpen algorithm selection and allocator warm-up, outside capture
                model.propagate_heads(*self.inputs)
        torch.cuda.current_stream(pred_init.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.outputs = model.propagate_heads(*self.inputs)

    def replay(self, pred_init=None, off_aff=None, confidence=None, dep=None) -> dict:
        for buf, new in zip(self.inputs, (pred_init, off_aff, confidence, dep)):
            if new is not None:
                buf.copy_(new)
        self.graph.replay()
        return self.outputs


def get(args):
    """Registry seam, src/model/__init__.py:17-22: model.get(args) -> model class."""
    if (args.model_name + "Model").lower() != "nlspnmodel":
        raise NotImplementedError(args.model_name)
    return NLSPNModel
