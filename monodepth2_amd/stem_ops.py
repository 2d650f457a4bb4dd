"""The ResNet stem convolution (conv1: 7x7, stride 2, padding 3, C -> 64, no bias) on
split-bf16 MFMA (csrc/stem.hip, ABI `md2_stem_*`): forward and weight gradient.

The stem reads the normalised frames, which are data: its backward is the weight
gradient alone, MIOpen's igemm_wrw at ~125 us (C=3, depth encoder, B=12) and ~430 us
(C=6, pose encoder, B=24) per step at 192x640.  stem_x6_wgrad_tr_kernel (f32-class:
three exact bf16 planes, six products; the window taps read from the staged rows with
transposing LDS reads) runs them in ~0.082 / ~0.21 ms including its split reduction
(tools/stem_bench.py; the earlier im2col-build kernel: ~0.10 / ~0.40 ms).  The forward
(MIOpen's igemm_fwd: 89 / 334 us) runs on stem_x6_fwd_kernel for C = 3 / 6 (the input
windows read straight from the NHWC rows as MFMA fragments, FWD_ENABLED).  Same
parameter (the torchvision `conv1.weight`), same semantics; any other case (an input
that needs a gradient, bf16, NCHW inputs, a CPU tensor) runs the module itself.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_CL = torch.channels_last
ENABLED = True       # the x6 weight gradient (tests flip it to compare with MIOpen)
FWD_ENABLED = os.environ.get("MD2_STEM_FWD", "1") != "0"   # the x6 forward (C = 3 / 6); 0: MIOpen's (A/B)
# bf16 autocast: the weight gradient on md2_stem_wgrad (deterministic) instead of MIOpen's bf16 one
BF16_ENABLED = os.environ.get("MD2_CONV_BF16", "1") != "0"


def _fwd(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """conv2d(x, weight, stride 2, padding 3) on md2_stem_fwd, or MIOpen's forward."""
    B, C, H, W = x.shape
    if not (FWD_ENABLED and C in (3, 6)):
        return F.conv2d(x, weight, None, 2, 3)
    w_cl = weight.is_contiguous(memory_format=_CL)
    if not (w_cl or weight.is_contiguous()):
        weight = weight.contiguous()
    d = _lib.StemDesc(B, C, H, W, _lib.STEM_WEIGHT_CL if w_cl else 0)
    y = torch.empty((B, 64, (H - 1) // 2 + 1, (W - 1) // 2 + 1), device=x.device, dtype=torch.float32,
                    memory_format=_CL)
    rc = _lib.lib().md2_stem_fwd(ctypes.byref(d), x.data_ptr(), weight.data_ptr(), y.data_ptr(), _lib.stream(x.device))
    _lib.check(rc, "md2_stem_fwd")
    return y


def _fwd_bf16(xb: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """The bf16 autocast stem convolution on md2_stem_fwd (MD2_STEM_BF16, ABI 23): bf16 x,
    the weight rounded to bf16 in the kernel, fp32 accumulation, bf16 y (C = 3 / 6)."""
    B, C, H, W = xb.shape
    w_cl = weight.is_contiguous(memory_format=_CL)
    if not (w_cl or weight.is_contiguous()):
        weight = weight.contiguous()
    d = _lib.StemDesc(B, C, H, W, (_lib.STEM_WEIGHT_CL if w_cl else 0) | _lib.STEM_BF16)
    y = torch.empty((B, 64, (H - 1) // 2 + 1, (W - 1) // 2 + 1), device=xb.device, dtype=torch.bfloat16,
                    memory_format=_CL)
    _lib.check(_lib.lib().md2_stem_fwd(ctypes.byref(d), xb.data_ptr(), weight.data_ptr(), y.data_ptr(),
                                       _lib.stream(xb.device)), "md2_stem_fwd")
    return y


_FWD_BF16 = os.environ.get("MD2_STEM_FWD_BF16", "1") != "0"   # A/B knob: 0 = MIOpen's bf16 forward


class _StemConv(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, weight):
        ctx.save_for_backward(x)
        ctx.w_cl = weight.is_contiguous(memory_format=_CL)
        ctx.w_shape = weight.shape
        return _fwd(x, weight)

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        gy = gy.contiguous(memory_format=_CL)
        B, C, H, W = x.shape
        d = _lib.StemDesc(B, C, H, W, _lib.STEM_WEIGHT_CL if ctx.w_cl else 0)
        gw = torch.empty(ctx.w_shape, device=x.device, dtype=torch.float32,
                         memory_format=_CL if ctx.w_cl else torch.contiguous_format)
        L = _lib.lib()
        ws = torch.empty(L.md2_stem_wgrad_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=x.device)
        rc = L.md2_stem_wgrad(ctypes.byref(d), x.data_ptr(), gy.data_ptr(), gw.data_ptr(), ws.data_ptr(),
                              _lib.stream(x.device))
        _lib.check(rc, "md2_stem_wgrad")
        return None, gw


_WGRAD_BF16 = os.environ.get("MD2_STEM_WGRAD_BF16", "1") != "0"   # A/B knob: 0 = fp32 copies of the operands


class _StemConvBF16(torch.autograd.Function):
    """The stem under bf16 autocast (config C5): the forward is autocast's arithmetic — x
    and the weight cast to bf16, fp32 accumulation, a bf16 output — on md2_stem_fwd's bf16
    form (C = 3 / 6; else MIOpen's bf16 convolution), and the weight gradient, which MIOpen
    computes non-deterministically in bf16, runs on md2_stem_wgrad (fixed-order reduction)
    over the bf16 operands themselves (MD2_STEM_BF16; C = 9: their exact fp32 values), then
    rounded to bf16 as the autocast cast's backward would hand it to the parameter."""

    @staticmethod
    def forward(ctx, x, weight):
        xb = x.to(torch.bfloat16)
        ctx.save_for_backward(xb)
        ctx.w_cl = weight.is_contiguous(memory_format=_CL)
        ctx.w_shape = weight.shape
        if _FWD_BF16 and FWD_ENABLED and xb.shape[1] in (3, 6) and xb.is_contiguous(memory_format=_CL):
            return _fwd_bf16(xb, weight)
        with torch.autocast("cuda", enabled=False):
            return F.conv2d(xb, weight.to(torch.bfloat16), None, 2, 3)

    @staticmethod
    def backward(ctx, gy):
        xb, = ctx.saved_tensors
        B, C, H, W = xb.shape
        flags = _lib.STEM_WEIGHT_CL if ctx.w_cl else 0
        if C in (3, 6) and gy.dtype == torch.bfloat16 and _WGRAD_BF16:
            # the bf16 operands as they are (MD2_STEM_BF16, ABI 23): one MFMA per fragment
            # pair instead of six with five zero planes, no fp32 copies — bitwise the same
            # sums (the zero planes add exact zeros; tests/test_stem_gpu.py)
            x = xb.contiguous(memory_format=_CL)
            gy = gy.contiguous(memory_format=_CL)
            flags |= _lib.STEM_BF16
        else:
            x = xb.float().contiguous(memory_format=_CL)
            gy = gy.float().contiguous(memory_format=_CL)
        d = _lib.StemDesc(B, C, H, W, flags)
        gw = torch.empty(ctx.w_shape, device=x.device, dtype=torch.float32,
                         memory_format=_CL if ctx.w_cl else torch.contiguous_format)
        L = _lib.lib()
        ws = torch.empty(L.md2_stem_wgrad_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=x.device)
        _lib.check(L.md2_stem_wgrad(ctypes.byref(d), x.data_ptr(), gy.data_ptr(), gw.data_ptr(), ws.data_ptr(),
                                    _lib.stream(x.device)), "md2_stem_wgrad")
        return None, gw.to(torch.bfloat16).to(torch.float32)


def supports_stem_bf16(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    from .conv_ops import _bf16_autocast
    return (BF16_ENABLED and x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32
            and not x.requires_grad and x.dim() == 4 and x.shape[1] in (3, 6, 9)
            and x.is_contiguous(memory_format=_CL) and conv.out_channels == 64
            and tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (3, 3)
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros" and _bf16_autocast() and x.numel() < 2 ** 31)


def supports_stem(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32 and not x.requires_grad
            and x.dim() == 4 and x.shape[1] in (3, 6, 9) and x.is_contiguous(memory_format=_CL)
            and conv.out_channels == 64 and tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2)
            and tuple(conv.padding) == (3, 3) and tuple(conv.dilation) == (1, 1) and conv.groups == 1
            and conv.bias is None and conv.padding_mode == "zeros" and not torch.is_autocast_enabled()
            and x.numel() < 2 ** 31)


def stem_conv(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """conv(x) for the encoder's stem; the weight gradient runs on md2_stem_wgrad when
    supports_stem(conv, x), else the module runs as is."""
    if ENABLED and supports_stem(conv, x):
        if torch.is_grad_enabled() and conv.weight.requires_grad:
            return _StemConv.apply(x, conv.weight)
        return _fwd(x, conv.weight.detach())
    if ENABLED and torch.is_grad_enabled() and conv.weight.requires_grad and supports_stem_bf16(conv, x):
        return _StemConvBF16.apply(x, conv.weight)
    return conv(x)
