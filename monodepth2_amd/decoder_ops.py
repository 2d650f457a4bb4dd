"""Fused DepthDecoder conv-input construction.

`conv_input(x, skip, elu, upsample)` = ReflectionPad2d(1)(cat([up(elu(x)), skip], 1))
in one HIP pass (md2_decoder_pad_fwd) with a one-pass adjoint (md2_decoder_pad_bwd).
Replaces the ELU / nearest-upsample / torch.cat / ReflectionPad2d chain of
networks/depth_decoder.py:50-65 + layers.py:106-136,196-199 between the MIOpen
convolutions.  GPU tensors only; `DepthDecoder` uses the eager chain on the CPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib


_CL = torch.channels_last


def _flags(elu: bool, upsample: bool, nhwc: bool, bf16: bool = False) -> int:
    return ((_lib.PAD_ELU if elu else 0) | (_lib.PAD_UPSAMPLE if upsample else 0) | (_lib.PAD_NHWC if nhwc else 0)
            | (_lib.PAD_BF16 if bf16 else 0))


class _ConvInput(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, skip, bias, elu: bool, upsample: bool, nhwc: bool, alias: bool = False):
        fmt = _CL if nhwc else torch.contiguous_format
        x = x.contiguous(memory_format=fmt)
        skip = skip.contiguous(memory_format=fmt) if skip is not None else None
        B, C, h, w = x.shape
        H, W = (2 * h, 2 * w) if upsample else (h, w)
        if skip is not None and tuple(skip.shape) != (B, skip.shape[1], H, W):
            raise ValueError(f"skip shape {tuple(skip.shape)} does not match {(B, '*', H, W)}")
        Cs = 0 if skip is None else skip.shape[1]
        out = torch.empty(B, C + Cs, H + 2, W + 2, device=x.device, dtype=x.dtype, memory_format=fmt)
        bf16 = x.dtype == torch.bfloat16
        if skip is not None and skip.dtype != x.dtype:
            skip = skip.to(x.dtype)
        d = _lib.PadDesc(B, C, h, w, Cs, _flags(elu, upsample, nhwc, bf16))
        bias32 = bias.detach().float().contiguous() if bias is not None else None
        rc = _lib.lib().md2_decoder_pad_fwd(ctypes.byref(d), x.data_ptr(),
                                            skip.data_ptr() if skip is not None else None,
                                            bias32.data_ptr() if bias32 is not None else None, out.data_ptr(),
                                            _lib.stream(x.device))
        _lib.check(rc, "md2_decoder_pad_fwd")
        ctx.elu, ctx.upsample, ctx.has_skip, ctx.nhwc, ctx.bf16 = elu, upsample, skip is not None, nhwc, bf16
        ctx.skip_shape = None if skip is None else skip.shape
        ctx.bias_dtype = None if bias is None else bias.dtype
        ctx.save_for_backward(x if elu else None, bias32)
        ctx.x_shape = x.shape
        if alias:   # (out, out') for out's two consumers; an unused one brings None
            ctx.set_materialize_grads(False)
            return out, out.view_as(out)
        return out

    @staticmethod
    def backward(ctx, gout, gout2=None):
        x, bias32 = ctx.saved_tensors
        fmt = _CL if ctx.nhwc else torch.contiguous_format
        if gout is None:
            gout, gout2 = gout2, None
        if gout is None:
            return None, None, None, None, None, None, None
        dt = torch.bfloat16 if ctx.bf16 else torch.float32
        gout = gout.to(dt).contiguous(memory_format=fmt)
        if gout2 is not None:
            gout2 = gout2.to(dt).contiguous(memory_format=fmt)
        B, C, h, w = ctx.x_shape
        gx = torch.empty(ctx.x_shape, device=gout.device, dtype=gout.dtype, memory_format=fmt)
        gskip = (torch.empty(ctx.skip_shape, device=gout.device, dtype=gout.dtype, memory_format=fmt)
                 if ctx.has_skip else None)
        d = _lib.PadDesc(B, C, h, w, 0 if gskip is None else ctx.skip_shape[1],
                         _flags(ctx.elu, ctx.upsample, ctx.nhwc, ctx.bf16))
        gbias = ws = None
        if bias32 is not None:
            gbias = torch.empty(C, device=gout.device, dtype=torch.float32)
            ws = torch.empty(_lib.lib().md2_decoder_pad_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                             device=gout.device)
        rc = _lib.lib().md2_decoder_pad_bwd2(ctypes.byref(d), x.data_ptr() if x is not None else None,
                                             bias32.data_ptr() if bias32 is not None else None,
                                             gout.data_ptr(), gout2.data_ptr() if gout2 is not None else None,
                                             gx.data_ptr(), gskip.data_ptr() if gskip is not None else None,
                                             gbias.data_ptr() if gbias is not None else None,
                                             ws.data_ptr() if ws is not None else None,
                                             _lib.stream(gout.device))
        _lib.check(rc, "md2_decoder_pad_bwd2")
        if gbias is not None and ctx.bias_dtype != torch.float32:
            gbias = gbias.to(ctx.bias_dtype)
        return gx, gskip, gbias, None, None, None, None


class _DispHead(torch.autograd.Function):
    """sigmoid(Conv2d(C, 1, 3)(P) + b) on the padded NHWC conv input (md2_disp_head_*)."""

    @staticmethod
    def forward(ctx, P, weight, bias):
        B, C, Hp, Wp = P.shape
        w_cl = weight.is_contiguous(memory_format=_CL)
        if not w_cl:
            weight = weight.contiguous()
        # bf16 P (config C5's bf16 decoder): read as is, its gradient written as bf16
        flags = (_lib.HEAD_WEIGHT_CL if w_cl else 0) | (_lib.HEAD_BF16 if P.dtype == torch.bfloat16 else 0)
        d = _lib.HeadDesc(B, C, Hp - 2, Wp - 2, flags)
        disp = torch.empty(B, 1, Hp - 2, Wp - 2, device=P.device, dtype=torch.float32)
        rc = _lib.lib().md2_disp_head_fwd(ctypes.byref(d), P.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                                          disp.data_ptr(), _lib.stream(P.device))
        _lib.check(rc, "md2_disp_head_fwd")
        ctx.d = d
        ctx.save_for_backward(P, weight, disp)
        return disp

    @staticmethod
    def backward(ctx, gdisp):
        P, weight, disp = ctx.saved_tensors
        d = ctx.d
        gdisp = gdisp.float().contiguous()
        gP = torch.empty_like(P, memory_format=_CL)   # P's dtype: bf16 input, bf16 gradient
        gw = torch.empty_like(weight)        # keeps the weight's memory format
        gb = torch.empty(1, device=P.device, dtype=torch.float32)
        ws = torch.empty(_lib.lib().md2_disp_head_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8,
                         device=P.device)
        rc = _lib.lib().md2_disp_head_bwd(ctypes.byref(d), P.data_ptr(), weight.data_ptr(), disp.data_ptr(),
                                          gdisp.data_ptr(), gP.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                                          ws.data_ptr(), _lib.stream(P.device))
        _lib.check(rc, "md2_disp_head_bwd")
        return gP, gw, gb


def supports_disp_head(P: torch.Tensor, conv: torch.nn.Conv2d, bf16_input: bool = False) -> bool:
    """The fused head takes fp32 NHWC inputs, one output channel, C % 4 == 0,
    C/4 dividing 256, C <= 256 (bf16_input: P is bf16, to be cast up by the caller)."""
    C = P.shape[1]
    want = torch.bfloat16 if bf16_input else torch.float32
    return (P.is_cuda and P.dtype == want and conv.weight.dtype == torch.float32
            and P.is_contiguous(memory_format=_CL) and conv.out_channels == 1 and conv.bias is not None
            and tuple(conv.kernel_size) == (3, 3) and tuple(conv.padding) == (0, 0)
            and tuple(conv.stride) == (1, 1) and C % 4 == 0 and C <= 256 and 256 % (C // 4) == 0)


def disp_head(P: torch.Tensor, conv: torch.nn.Conv2d) -> torch.Tensor:
    """sigmoid(conv(P)) for the decoder's Conv2d(C, 1, 3) disparity head in one HIP
    pass each way (networks/depth_decoder.py:63-64 dispconv + sigmoid).  P fp32, or bf16
    (config C5: read as is, fp32 arithmetic and weights, fp32 disparities)."""
    if not supports_disp_head(P, conv, bf16_input=P.dtype == torch.bfloat16):
        raise ValueError("disp_head: fp32 / bf16 channels_last input, Conv2d(C, 1, 3) with bias, C/4 dividing 256")
    return _DispHead.apply(P, conv.weight, conv.bias)


_POSE_MIOPEN = os.environ.get("MD2_POSE_MIOPEN", "0") == "1"   # A/B knob: the pose decoder's convs on MIOpen


class _BiasAct(torch.autograd.Function):
    """[relu](z + b) in place on the convolution's own output z, one HIP pass each way
    (md2_bias_act_*); z's gradient goes back to the convolution's backward."""

    @staticmethod
    def forward(ctx, z, bias, relu: bool):
        B, C, H, W = z.shape
        d = _lib.BiasActDesc(B * H * W, C, _lib.BIAS_ACT_RELU if relu else 0)
        _lib.check(_lib.lib().md2_bias_act_fwd(ctypes.byref(d), z.data_ptr(), bias.data_ptr(), z.data_ptr(),
                                               _lib.stream(z.device)),
                   "md2_bias_act_fwd")                      # in place: z is the convolution's fresh output
        ctx.mark_dirty(z)
        ctx.save_for_backward(z if relu else None)
        ctx.conf = (relu, d)
        return z

    @staticmethod
    def backward(ctx, gy):
        y, = ctx.saved_tensors
        relu, d = ctx.conf
        gy = gy.contiguous(memory_format=_CL)
        gb = torch.empty(gy.shape[1], device=gy.device, dtype=torch.float32)
        gz = torch.empty_like(gy, memory_format=_CL) if relu else gy
        L = _lib.lib()
        ws = torch.empty(L.md2_bias_act_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=gy.device)
        _lib.check(L.md2_bias_act_bwd(ctypes.byref(d), y.data_ptr() if relu else None, gy.data_ptr(),
                                      gz.data_ptr() if relu else None, gb.data_ptr(), ws.data_ptr(),
                                      _lib.stream(gy.device)),
                   "md2_bias_act_bwd")
        return gz, gb, None


class _BiasActBF16(torch.autograd.Function):
    """[relu](z + bf16(b)) for config C5's bf16 pose decoder, autocast's arithmetic forward
    (one bf16 add, the ReLU); backward on md2_bias_act_bwd over the exact fp32 widening of
    the bf16 operands: the ReLU mask (bitwise torch's threshold_backward on the bf16 values)
    and the bias gradient as a fixed-order fp32 sum, rounded to bf16 as autocast's bf16 sum
    leaves it.  The bias gradient was ATen's bf16 sum before: inside C5's captured step its
    value changed between replays of one state (~20 of pose_0's 256 channels by one bf16
    ulp, 1 replay in 2; tools/c5_replay_diag.py), the only non-repeatable gradient there."""

    @staticmethod
    def forward(ctx, z, bias, relu: bool):
        y = z + bias.to(torch.bfloat16).view(1, -1, 1, 1)
        if relu:
            y = torch.relu(y)
        ctx.save_for_backward(y if relu else None)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, gy):
        y, = ctx.saved_tensors
        relu = ctx.relu
        B, C, H, W = gy.shape
        g32 = gy.float().contiguous(memory_format=_CL)
        y32 = y.float().contiguous(memory_format=_CL) if relu else None
        d = _lib.BiasActDesc(B * H * W, C, _lib.BIAS_ACT_RELU if relu else 0)
        gb = torch.empty(C, device=gy.device, dtype=torch.float32)
        gz32 = torch.empty_like(g32, memory_format=_CL) if relu else None
        L = _lib.lib()
        ws = torch.empty(L.md2_bias_act_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=gy.device)
        _lib.check(L.md2_bias_act_bwd(ctypes.byref(d), y32.data_ptr() if relu else None, g32.data_ptr(),
                                      gz32.data_ptr() if relu else None, gb.data_ptr(), ws.data_ptr(),
                                      _lib.stream(gy.device)), "md2_bias_act_bwd")
        gz = gz32.to(torch.bfloat16) if relu else gy
        return gz, gb.to(torch.bfloat16).float(), None


_BF16_BIAS_ACT = os.environ.get("MD2_BF16_BIAS_ACT", "1") != "0"   # A/B knob: 0 = ATen's add / relu / sum


def conv_bias_act(conv: torch.nn.Conv2d, x: torch.Tensor, relu: bool) -> torch.Tensor:
    """relu?(conv(x)) for the pose decoder (networks/pose_decoder.py:43-54): the
    convolution bias-free on conv_ops (split-bf16 MFMA kernels chosen per shape against
    MIOpen, forward and both gradients), the bias (+ ReLU) as one HIP pass each way, when
    x is a CUDA fp32 channels_last tensor; else eager."""
    if (x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32 and conv.bias is not None
            and x.is_contiguous(memory_format=_CL) and conv.weight.is_contiguous(memory_format=_CL)
            and conv.out_channels % 4 == 0 and conv.groups == 1 and tuple(conv.dilation) == (1, 1)
            and conv.padding_mode == "zeros" and not torch.is_autocast_enabled() and torch.is_grad_enabled()
            and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]):
        from .conv_ops import conv2d_w
        z = (F.conv2d(x, conv.weight, None, conv.stride, conv.padding) if _POSE_MIOPEN
             else conv2d_w(x, conv.weight, conv.stride[0], conv.padding[0]))
        if not z.is_contiguous(memory_format=_CL):
            z = z.contiguous(memory_format=_CL)
        return _BiasAct.apply(z, conv.bias, relu)
    from . import conv_ops
    if (conv.bias is not None and conv.groups == 1 and tuple(conv.dilation) == (1, 1) and conv.padding_mode == "zeros"
            and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
            and conv_ops._bf16_ok(x, conv.weight, conv.stride[0], conv.padding[0])):
        # bf16 autocast (config C5): the bias-free bf16 convolution (conv_ops.conv2d_bf16,
        # deterministic weight gradient), the bf16-cast bias added as autocast's conv
        # would, then the ReLU
        z = conv_ops.conv2d_bf16(x, conv.weight, conv.stride[0], conv.padding[0])
        if _BF16_BIAS_ACT and z.is_contiguous(memory_format=_CL) and conv.out_channels % 4 == 0:
            return _BiasActBF16.apply(z, conv.bias, relu)
        z = z + conv.bias.to(torch.bfloat16).view(1, -1, 1, 1)
        return F.relu(z) if relu else z
    y = conv(x)
    return F.relu(y) if relu else y


def supports_bf16(x: torch.Tensor, skip: Optional[torch.Tensor], nhwc: bool) -> bool:
    return nhwc and x.shape[1] % 4 == 0 and (skip is None or skip.shape[1] % 4 == 0)


def supports_bias(channels: int, nhwc: bool) -> bool:
    """A conv bias over `channels` can be folded into conv_input (NHWC, C/4 dividing 256)."""
    return nhwc and channels % 4 == 0 and 256 % (channels // 4) == 0


# A/B knob: MD2_ALIAS_SUM=0 leaves a shared padded map's two gradients to autograd's add
ALIAS_SUM = os.environ.get("MD2_ALIAS_SUM", "1") != "0"


def conv_input(x: torch.Tensor, skip: Optional[torch.Tensor] = None, elu: bool = False,
               upsample: bool = False, nhwc: bool = False, bias: Optional[torch.Tensor] = None,
               alias: bool = False):
    """ReflectionPad2d(1)(cat([upsample?(elu?(x + bias)), skip], 1)) in one fused pass.
    nhwc: tensors in (and out) channels_last, as the NHWC convolutions around it.
    bias: the bias of the conv that produced x (that conv then runs without one);
    its gradient comes back from the same backward pass.
    alias: returns (P, P') with P' a view of P for its second consumer (dispconv beside
    the next level's conv); in NHWC with channel counts multiple of 4 the two gradients
    are summed as the backward reads them (md2_decoder_pad_bwd2), else P' is P."""
    if x.device.type != "cuda":
        raise RuntimeError("conv_input is a HIP kernel; use the eager chain on the CPU")
    if x.dtype != torch.float32 and not (x.dtype == torch.bfloat16 and supports_bf16(x, skip, nhwc)):
        raise ValueError("conv_input supports float32, and bfloat16 in NHWC with channel counts multiple of 4")
    if bias is not None and not supports_bias(x.shape[1], nhwc):
        raise ValueError("conv_input folds a bias only in NHWC with C/4 dividing 256")
    if alias:
        sc = 0 if skip is None else skip.shape[1]
        if ALIAS_SUM and nhwc and x.shape[1] % 4 == 0 and sc % 4 == 0 and torch.is_grad_enabled():
            return _ConvInput.apply(x, skip, bias, elu, upsample, nhwc, True)
        P = _ConvInput.apply(x, skip, bias, elu, upsample, nhwc, False)
        return P, P
    return _ConvInput.apply(x, skip, bias, elu, upsample, nhwc, False)
