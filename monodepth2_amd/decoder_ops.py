"""Fused DepthDecoder conv-input construction.

`conv_input(x, skip, elu, upsample)` = ReflectionPad2d(1)(cat([up(elu(x)), skip], 1))
in one HIP pass (md2_decoder_pad_fwd) with a one-pass adjoint (md2_decoder_pad_bwd).
Replaces the ELU / nearest-upsample / torch.cat / ReflectionPad2d chain of
networks/depth_decoder.py:50-65 + layers.py:106-136,196-199 between the MIOpen
convolutions.  GPU tensors only; `DepthDecoder` uses the eager chain on the CPU.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib


def _desc(x: torch.Tensor, skip: Optional[torch.Tensor], elu: bool, upsample: bool) -> _lib.PadDesc:
    B, C, h, w = x.shape
    return _lib.PadDesc(B, C, h, w, 0 if skip is None else skip.shape[1],
                        (_lib.PAD_ELU if elu else 0) | (_lib.PAD_UPSAMPLE if upsample else 0))


class _ConvInput(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, skip, elu: bool, upsample: bool):
        x = x.contiguous()
        skip = skip.contiguous() if skip is not None else None
        B, C, h, w = x.shape
        H, W = (2 * h, 2 * w) if upsample else (h, w)
        if skip is not None and tuple(skip.shape) != (B, skip.shape[1], H, W):
            raise ValueError(f"skip shape {tuple(skip.shape)} does not match {(B, '*', H, W)}")
        Cs = 0 if skip is None else skip.shape[1]
        out = torch.empty(B, C + Cs, H + 2, W + 2, device=x.device, dtype=x.dtype)
        d = _desc(x, skip, elu, upsample)
        rc = _lib.lib().md2_decoder_pad_fwd(ctypes.byref(d), x.data_ptr(),
                                            skip.data_ptr() if skip is not None else None, out.data_ptr(),
                                            torch.cuda.current_stream(x.device).cuda_stream)
        _lib.check(rc, "md2_decoder_pad_fwd")
        ctx.elu, ctx.upsample, ctx.has_skip = elu, upsample, skip is not None
        ctx.skip_shape = None if skip is None else skip.shape
        ctx.save_for_backward(x if elu else None)
        ctx.x_shape = x.shape
        return out

    @staticmethod
    def backward(ctx, gout):
        (x,) = ctx.saved_tensors
        gout = gout.contiguous()
        B, C, h, w = ctx.x_shape
        gx = torch.empty(ctx.x_shape, device=gout.device, dtype=gout.dtype)
        gskip = torch.empty(ctx.skip_shape, device=gout.device, dtype=gout.dtype) if ctx.has_skip else None
        d = _lib.PadDesc(B, C, h, w, 0 if gskip is None else ctx.skip_shape[1],
                         (_lib.PAD_ELU if ctx.elu else 0) | (_lib.PAD_UPSAMPLE if ctx.upsample else 0))
        rc = _lib.lib().md2_decoder_pad_bwd(ctypes.byref(d), x.data_ptr() if x is not None else None,
                                            gout.data_ptr(), gx.data_ptr(),
                                            gskip.data_ptr() if gskip is not None else None,
                                            torch.cuda.current_stream(gout.device).cuda_stream)
        _lib.check(rc, "md2_decoder_pad_bwd")
        return gx, gskip, None, None


def conv_input(x: torch.Tensor, skip: Optional[torch.Tensor] = None, elu: bool = False,
               upsample: bool = False) -> torch.Tensor:
    """ReflectionPad2d(1)(cat([upsample?(elu?(x)), skip], 1)) in one fused pass."""
    if x.device.type != "cuda":
        raise RuntimeError("conv_input is a HIP kernel; use the eager chain on the CPU")
    if x.dtype != torch.float32:
        raise ValueError("conv_input supports float32")
    return _ConvInput.apply(x, skip, elu, upsample)
