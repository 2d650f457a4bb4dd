"""ResNet encoder without torchvision (torchvision is not installed here).

Same public API as the reference `networks/resnet_encoder.py:62-98`
(`ResnetEncoder(num_layers, pretrained, num_input_images=1)`, `.num_ch_enc`,
forward -> five feature maps) and the same parameter names as torchvision's
ResNet (`encoder.conv1.weight`, `encoder.layer1.0.bn1.running_mean`,
`encoder.fc.weight`, ...), so checkpoints interchange with the reference.

Weight init follows torchvision / `resnet_encoder.py:34-39`: Kaiming-normal
(fan_out, relu) convolutions, BN weight 1 / bias 0.  ImageNet weights
(`pretrained=True`, `resnet_encoder.py:54-58`) need the network and are not
available offline: requesting them warns and keeps the random init.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch
import torch.nn as nn

from ..bn_ops import bn_act, max_pool_3x3s2, max_pool_3x3s2_with_alias
from ..conv_ops import conv2d
from ..stem_ops import stem_conv


def _conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # relu(bn(conv)) and relu(bn(conv) + identity), fused on the GPU (bn_ops)
        identity = x if self.downsample is None else _downsample(self.downsample, x)
        out = bn_act(self.bn1, self.conv1(x))
        return bn_act(self.bn2, self.conv2(out), residual=identity)


def _downsample(down: nn.Sequential, x):
    """The (conv1x1, BatchNorm2d) shortcut: BN without ReLU."""
    return bn_act(down[1], conv2d(down[0], x), relu=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = _conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = _conv1x1(planes, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else _downsample(self.downsample, x)
        out = bn_act(self.bn1, self.conv1(x))
        out = bn_act(self.bn2, self.conv2(out))
        return bn_act(self.bn3, self.conv3(out), residual=identity)


def _run_layer(layer: nn.Sequential, x, xs, skip_alias: bool):
    """The blocks of one ResNet stage (torchvision BasicBlock / Bottleneck semantics)
    with each block output handed out as views for its other consumers — the next
    block's shortcut and, for the stage output, the decoder skip — so the fused
    BatchNorm backward sums their gradients on load (bn_act aliases) instead of
    autograd adding them.  x feeds the block's first conv, xs (the same values) its
    shortcut.  Returns (output, its shortcut view, its skip view)."""
    n = len(layer)
    skip = None
    for bi, blk in enumerate(layer):
        shortcut = xs if blk.downsample is None else _downsample(blk.downsample, xs)
        out = bn_act(blk.bn1, conv2d(blk.conv1, x))
        if isinstance(blk, Bottleneck):
            out = bn_act(blk.bn2, conv2d(blk.conv2, out))
            bn, conv = blk.bn3, blk.conv3
        else:
            bn, conv = blk.bn2, blk.conv2
        last = bi == n - 1
        k = (2 if skip_alias else 1) if last else 1
        res = bn_act(bn, conv2d(conv, out), residual=shortcut, aliases=k)
        x, xs = res[0], res[1]
        skip = res[2] if (last and skip_alias) else x
    return x, xs, skip


_SPECS = {18: (BasicBlock, [2, 2, 2, 2]), 34: (BasicBlock, [3, 4, 6, 3]), 50: (Bottleneck, [3, 4, 6, 3]),
          101: (Bottleneck, [3, 4, 23, 3]), 152: (Bottleneck, [3, 8, 36, 3])}


class ResNet(nn.Module):
    """torchvision-layout ResNet trunk (+ unused avgpool/fc kept for key parity)."""

    def __init__(self, num_layers=18, in_channels=3, num_classes=1000):
        super().__init__()
        block, counts = _SPECS[num_layers]
        self.inplanes = 64
        self.conv1 = nn.Conv2d(in_channels, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._stage(block, 64, counts[0])
        self.layer2 = self._stage(block, 128, counts[1], stride=2)
        self.layer3 = self._stage(block, 256, counts[2], stride=2)
        self.layer4 = self._stage(block, 512, counts[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _stage(self, block, planes, n, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(_conv1x1(self.inplanes, planes * block.expansion, stride),
                                 nn.BatchNorm2d(planes * block.expansion))
        blocks = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        blocks += [block(self.inplanes, planes) for _ in range(1, n)]
        return nn.Sequential(*blocks)


class ResnetEncoder(nn.Module):
    """Pytorch module for a resnet encoder (resnet_encoder.py:62-98)."""

    def __init__(self, num_layers, pretrained, num_input_images=1):
        super().__init__()
        if num_layers not in _SPECS:
            raise ValueError("{} is not a valid number of resnet layers".format(num_layers))
        if num_input_images > 1 and num_layers not in (18, 50):
            raise AssertionError("Can only run with 18 or 50 layer resnet")
        if pretrained:
            warnings.warn("ImageNet weights need network access and are unavailable offline; "
                          "using the random (scratch) initialisation instead")
        self.num_ch_enc = np.array([64, 64, 128, 256, 512])
        self.encoder = ResNet(num_layers, in_channels=3 * num_input_images)
        if num_layers > 34:
            self.num_ch_enc[1:] *= 4

    MEAN, STD = 0.45, 0.225   # resnet_encoder.py:93

    def prepare(self, frames):
        """The normalised encoder input.  frames: a (B,3,H,W) tensor, or a list of
        frame pairs [[(B,3,H,W), (B,3,H,W)], ...] concatenated along channels (pose
        encoder, trainer.py:280-290) and along the batch.  On the GPU with NHWC
        convolutions: one HIP pass straight into channels_last (md2_encoder_input)."""
        groups = [[frames]] if torch.is_tensor(frames) else [list(p) for p in frames]
        f0 = groups[0][0]
        if (f0.is_cuda and f0.dtype == torch.float32 and f0.dim() == 4 and f0.shape[1] == 3
                and self.encoder.conv1.weight.is_contiguous(memory_format=torch.channels_last)
                and len(groups) * len(groups[0]) <= 8
                and all(t.shape == f0.shape and t.dtype == f0.dtype and t.is_contiguous() for g in groups for t in g)):
            import ctypes
            from .. import _lib
            B, _, H, W = f0.shape
            S = len(groups[0])
            out = torch.empty(len(groups) * B, 3 * S, H, W, device=f0.device, memory_format=torch.channels_last)
            src = (ctypes.c_void_p * (len(groups) * S))(*[t.data_ptr() for g in groups for t in g])
            rc = _lib.lib().md2_encoder_input(len(groups), B, S, H, W, src, self.MEAN, self.STD, out.data_ptr(),
                                              torch.cuda.current_stream(f0.device).cuda_stream)
            _lib.check(rc, "md2_encoder_input")
            return out
        x = torch.cat([torch.cat(g, 1) for g in groups], 0) if len(groups) * len(groups[0]) > 1 else f0
        x = (x - self.MEAN) / self.STD
        if self.encoder.conv1.weight.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        return x

    def forward(self, input_image):
        return self.forward_prepared(self.prepare(input_image))

    def forward_prepared(self, x):
        """The encoder on an input already normalised by `prepare`."""
        e = self.encoder
        f0 = bn_act(e.bn1, stem_conv(e.conv1, x))   # weight gradient on f32 MFMA (stem_ops)
        # f0's two gradients (layer1, decoder skip) and the pooled map's two (the first
        # block's conv1 and shortcut) all meet in the pool backward
        x, xs, f0 = max_pool_3x3s2_with_alias(e.maxpool, f0, out_alias=True)
        feats = [f0]
        layers = [e.layer1, e.layer2, e.layer3, e.layer4]
        for li, layer in enumerate(layers):
            # every layer output but the last also feeds the decoder skip
            x, xs, skip = _run_layer(layer, x, xs, skip_alias=li < len(layers) - 1)
            feats.append(skip)
        self.features = feats
        return self.features
