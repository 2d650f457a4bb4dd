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

from ..bn_ops import bn_act, max_pool_3x3s2


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
    return bn_act(down[1], down[0](x), relu=False)


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

    def forward(self, input_image):
        e = self.encoder
        x = (input_image - 0.45) / 0.225
        if e.conv1.weight.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        f0 = bn_act(e.bn1, e.conv1(x))
        f1 = e.layer1(max_pool_3x3s2(e.maxpool, f0))
        f2 = e.layer2(f1)
        f3 = e.layer3(f2)
        f4 = e.layer4(f3)
        self.features = [f0, f1, f2, f3, f4]
        return self.features
