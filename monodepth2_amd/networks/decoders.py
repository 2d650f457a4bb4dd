"""Depth and pose decoders (PyTorch-ROCm modules; convolutions run on MIOpen).

Restates `networks/depth_decoder.py:14-65`, `networks/pose_decoder.py:14-54` and
`networks/pose_cnn.py:14-50` with identical constructor signatures, forward
outputs and parameter names (`decoder.{i}.conv.conv.weight`, `net.{i}.weight`),
so reference checkpoints load unchanged.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..layers import Conv3x3, ConvBlock, upsample

import os

# bf16 autocast: the disparity heads on the fused fp32 head kernels (A/B knob: 0 = the
# module under autocast, i.e. MIOpen's bf16 convolution + sigmoid)
_AMP_HEADS = os.environ.get("MD2_AMP_FUSED_HEADS", "1") != "0"


class DepthDecoder(nn.Module):
    """5-level skip decoder with sigmoid disparity heads (depth_decoder.py:14-65).

    Module order inside `decoder` (state-dict indices): for i = 4..0 the pair
    (upconv i 0, upconv i 1), then one dispconv per scale.
    """

    def __init__(self, num_ch_enc, scales=range(4), num_output_channels=1, use_skips=True):
        super().__init__()
        self.num_output_channels = num_output_channels
        self.use_skips = use_skips
        self.upsample_mode = "nearest"
        self.scales = scales
        self.num_ch_enc = num_ch_enc
        self.num_ch_dec = np.array([16, 32, 64, 128, 256])
        ch_enc, ch_dec = self.num_ch_enc, self.num_ch_dec
        self.convs = {}
        mods = []
        for i in range(4, -1, -1):
            cin = ch_enc[-1] if i == 4 else ch_dec[i + 1]
            self.convs[("upconv", i, 0)] = ConvBlock(cin, ch_dec[i])
            cin = ch_dec[i] + (ch_enc[i - 1] if (use_skips and i > 0) else 0)
            self.convs[("upconv", i, 1)] = ConvBlock(cin, ch_dec[i])
            mods += [self.convs[("upconv", i, 0)], self.convs[("upconv", i, 1)]]
        for s in self.scales:
            self.convs[("dispconv", s)] = Conv3x3(ch_dec[s], num_output_channels)
            mods.append(self.convs[("dispconv", s)])
        self.decoder = nn.ModuleList(mods)
        self.sigmoid = nn.Sigmoid()
        self.fused = True   # GPU: build each conv input with the fused HIP pass
        self.fused_heads = True   # GPU fp32: dispconv + sigmoid as one HIP pass (decoder_ops.disp_head)

    def _forward_fused(self, input_features):
        """Same graph with each conv input built by one HIP pass (decoder_ops):
        pad(x) -> conv -> [ELU -> up x2 -> cat skip -> pad] -> conv -> [ELU -> pad] ->
        (dispconv -> sigmoid) and the next level's first conv."""
        from ..conv_ops import conv2d_w
        from ..decoder_ops import conv_input, disp_head, supports_bias, supports_disp_head
        self.outputs = {}
        # NHWC convolutions (channels_last weights): keep every conv input NHWC too
        cl = self.convs[("upconv", 4, 0)].conv.conv.weight.is_contiguous(memory_format=torch.channels_last)
        P = conv_input(input_features[-1], nhwc=cl)               # ReflectionPad2d only

        def conv(block, P):
            """The block's conv; its bias moves into the next conv_input when that can
            fold it (NHWC: no separate bias-add pass forward, no bias-grad reduction
            backward — the pad kernels carry both)."""
            c = block.conv.conv
            if c.bias is not None and supports_bias(c.out_channels, cl) and c.groups == 1 \
                    and tuple(c.dilation) == (1, 1) and c.stride[0] == c.stride[1] and c.padding[0] == c.padding[1]:
                # f32 MFMA implicit GEMM where the channel counts fit (conv_ops), else MIOpen
                return conv2d_w(P, c.weight, c.stride[0], c.padding[0]), c.bias
            return c(P), None

        for i in range(4, -1, -1):
            y0, b0 = conv(self.convs[("upconv", i, 0)], P)
            skip = input_features[i - 1] if (self.use_skips and i > 0) else None
            P = conv_input(y0, skip, elu=True, upsample=True, nhwc=cl, bias=b0)
            y1, b1 = conv(self.convs[("upconv", i, 1)], P)
            if i in self.scales and i > 0:   # shared by dispconv and the next level: a view each,
                P, Ph = conv_input(y1, None, elu=True, upsample=False, nhwc=cl, bias=b1, alias=True)
            else:                            # their gradients summed in the pad backward
                P = Ph = conv_input(y1, None, elu=True, upsample=False, nhwc=cl, bias=b1)
            if i in self.scales:
                head = self.convs[("dispconv", i)].conv
                if self.fused_heads and supports_disp_head(Ph, head) and not torch.is_autocast_enabled():
                    self.outputs[("disp", i)] = disp_head(Ph, head)
                elif (self.fused_heads and _AMP_HEADS and torch.is_autocast_enabled()
                        and supports_disp_head(Ph, head, bf16_input=True)):
                    # bf16 autocast (config C5): the same fused head reading the bf16 input
                    # (widened exactly; fp32 weight and arithmetic, fp32 disparities, a bf16
                    # input gradient) — instead of MIOpen's C -> 1 bf16 convolution + a
                    # separate sigmoid each way
                    with torch.autocast("cuda", enabled=False):
                        self.outputs[("disp", i)] = disp_head(Ph, head)
                else:
                    self.outputs[("disp", i)] = self.sigmoid(head(Ph))
        return self.outputs

    def forward(self, input_features):
        f = input_features[-1]
        cl = self.convs[("upconv", 4, 0)].conv.conv.weight.is_contiguous(memory_format=torch.channels_last)
        if (f.is_cuda and self.fused and self.num_output_channels >= 1
                and (f.dtype == torch.float32 or (f.dtype == torch.bfloat16 and cl))):   # bf16: NHWC kernels
            return self._forward_fused(input_features)
        self.outputs = {}
        x = input_features[-1]
        for i in range(4, -1, -1):
            x = upsample(self.convs[("upconv", i, 0)](x))
            if self.use_skips and i > 0:
                x = torch.cat([x, input_features[i - 1]], 1)
            x = self.convs[("upconv", i, 1)](x)
            if i in self.scales:
                self.outputs[("disp", i)] = self.sigmoid(self.convs[("dispconv", i)](x))
        return self.outputs


class PoseDecoder(nn.Module):
    """Pose head: squeeze + 3 convs + spatial mean, scaled by 0.01 (pose_decoder.py:14-54)."""

    def __init__(self, num_ch_enc, num_input_features, num_frames_to_predict_for=None, stride=1):
        super().__init__()
        self.num_ch_enc = num_ch_enc
        self.num_input_features = num_input_features
        if num_frames_to_predict_for is None:
            num_frames_to_predict_for = num_input_features - 1
        self.num_frames_to_predict_for = num_frames_to_predict_for
        self.convs = {
            "squeeze": nn.Conv2d(self.num_ch_enc[-1], 256, 1),
            ("pose", 0): nn.Conv2d(num_input_features * 256, 256, 3, stride, 1),
            ("pose", 1): nn.Conv2d(256, 256, 3, stride, 1),
            ("pose", 2): nn.Conv2d(256, 6 * num_frames_to_predict_for, 1),
        }
        self.relu = nn.ReLU()
        self.net = nn.ModuleList([self.convs["squeeze"], self.convs[("pose", 0)], self.convs[("pose", 1)],
                                  self.convs[("pose", 2)]])
        # True: forward returns the packed (N, frames, 1, 6) [axisangle | translation]
        # tensor instead of its two slices (the trainer's fused pose producer reads it
        # whole; one gradient tensor comes back instead of two slice adjoints)
        self.packed_output = False

    def forward(self, input_features):
        from ..decoder_ops import conv_bias_act   # bias (+ ReLU) as one HIP pass each way on the GPU
        sq = [conv_bias_act(self.convs["squeeze"], f[-1], True) for f in input_features]
        x = torch.cat(sq, 1) if len(sq) > 1 else sq[0]
        x = conv_bias_act(self.convs[("pose", 0)], x, True)
        x = conv_bias_act(self.convs[("pose", 1)], x, True)
        x = conv_bias_act(self.convs[("pose", 2)], x, False)
        x = 0.01 * x.mean(3).mean(2).view(-1, self.num_frames_to_predict_for, 1, 6)
        if self.packed_output:
            return x
        return x[..., :3], x[..., 3:]


class PoseCNN(nn.Module):
    """Stand-alone pose network of Zhou et al. (pose_cnn.py:14-50)."""

    def __init__(self, num_input_frames):
        super().__init__()
        self.num_input_frames = num_input_frames
        spec = [(3 * num_input_frames, 16, 7, 3), (16, 32, 5, 2), (32, 64, 3, 1), (64, 128, 3, 1),
                (128, 256, 3, 1), (256, 256, 3, 1), (256, 256, 3, 1)]
        self.convs = {i: nn.Conv2d(cin, cout, k, 2, p) for i, (cin, cout, k, p) in enumerate(spec)}
        self.pose_conv = nn.Conv2d(256, 6 * (num_input_frames - 1), 1)
        self.num_convs = len(self.convs)
        self.relu = nn.ReLU(True)
        self.net = nn.ModuleList([self.convs[i] for i in range(self.num_convs)])

    def forward(self, out):
        for i in range(self.num_convs):
            out = self.relu(self.convs[i](out))
        out = self.pose_conv(out).mean(3).mean(2)
        out = 0.01 * out.view(-1, self.num_input_frames - 1, 1, 6)
        return out[..., :3], out[..., 3:]
