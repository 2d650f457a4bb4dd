"""Fused training-mode BatchNorm2d (+ residual add) (+ ReLU) for the ResNet encoders
(csrc/bnorm.hip, ABI `md2_bn_*`).

`bn_act(bn, x, residual, relu)` computes relu(bn(x) [+ residual]) for an
`nn.BatchNorm2d` module with its own parameters and buffers (so the torchvision
state-dict keys of networks/resnet_encoder.py are unchanged): two HIP launches
forward, two backward, instead of MIOpen's three-kernel BatchNorm each way plus the
separate ReLU / add passes.  It takes the channels_last (NHWC) activations of the
default build, fp32 or bf16 (--amp bf16: bf16 storage, fp32 arithmetic and
statistics); other layouts, eval mode, momentum=None and the CPU run
`nn.BatchNorm2d` itself.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

ENABLED = True   # tests flip this to compare with nn.BatchNorm2d on the same module
_GROUPS = 1      # bn_groups(): the batch holds this many independently normalised chunks


@contextlib.contextmanager
def bn_groups(n: int):
    """Inside, every bn_act treats its batch as n equal consecutive chunks with their
    own batch statistics — identical to running the network on each chunk separately
    (convolutions, pooling and activations are per-image anyway).  The trainer runs
    the pose encoder once over both frame pairs this way."""
    global _GROUPS
    prev, _GROUPS = _GROUPS, int(n)
    try:
        yield
    finally:
        _GROUPS = prev

_CL = torch.channels_last
_workspaces: Dict[int, torch.Tensor] = {}
_workspaces_keep = []


def _workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Scratch (partial sums + backward coefficients) per HIP stream: calls on one
    stream are ordered, calls on different streams (the trainer runs the pose
    network beside the depth network) must not share it."""
    key = _lib.stream(device)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() < nbytes:
        if ws is not None:   # never freed: a captured hipGraph may still use it (conv_ops._workspace)
            _workspaces_keep.append(ws)
        with torch.cuda.stream(torch.cuda.current_stream(device)):
            ws = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _workspaces[key] = ws
    return ws


_descs: Dict[tuple, tuple] = {}


def _desc(key: tuple):
    """(BnDesc, workspace bytes) per (pixels, C, flags, eps, momentum, groups): built once,
    the ~80 calls per step reuse them (the step is close to launch-bound)."""
    hit = _descs.get(key)
    if hit is None:
        d = _lib.BnDesc(*key, 0)
        hit = _descs[key] = (d, _lib.lib().md2_bn_workspace_bytes(ctypes.byref(d)))
    return hit


def _supported(C: int) -> bool:
    """Channel counts the kernels take: C/4 a power of two (every ResNet width)."""
    Q = C // 4
    return C % 4 == 0 and Q > 0 and (Q & (Q - 1)) == 0


class _BNAct(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, relu: bool, eps: float,
                momentum: float, groups: int, aliases: int = 0):
        B, C, H, W = x.shape
        flags = ((_lib.BN_RELU if relu else 0) | (_lib.BN_RESIDUAL if residual is not None else 0)
                 | (_lib.BN_BF16 if x.dtype == torch.bfloat16 else 0))
        key = (B * H * W, C, flags, eps, momentum, groups)
        d, nbytes = _desc(key)
        L = _lib.lib()
        ws = _workspace(x.device, nbytes)
        y = torch.empty_like(x, memory_format=_CL)
        stats = torch.empty(2, groups, C, device=x.device)   # saved mean, invstd
        mean, invstd = stats[0], stats[1]
        # with ReLU the backward needs only y > 0: one mask byte per element quad (ABI 15)
        mask = torch.empty(x.numel() // 4, dtype=torch.uint8, device=x.device) if relu else None
        stream = _lib.stream(x.device)
        rc = L.md2_bn_fwd_mask(ctypes.byref(d), x.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                               residual.data_ptr() if residual is not None else None,
                               running_mean.data_ptr() if running_mean is not None else None,
                               running_var.data_ptr() if running_var is not None else None,
                               y.data_ptr(), mask.data_ptr() if mask is not None else None,
                               mean.data_ptr(), invstd.data_ptr(), ws.data_ptr(), stream)
        _lib.check(rc, "md2_bn_fwd_mask")
        ctx.save_for_backward(x, mask, weight, mean, invstd)
        ctx.desc = key
        ctx.has_res = residual is not None
        if aliases:
            # views of y for its other consumers: their gradients come into this backward
            # and are summed on load by the backward kernels (md2_bn_bwd_multi)
            ctx.set_materialize_grads(False)
            return (y,) + tuple(y.view_as(y) for _ in range(aliases))
        return y

    @staticmethod
    def backward(ctx, *grads):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        gs = [g.to(x.dtype).contiguous(memory_format=_CL) for g in grads if g is not None]
        if not gs:
            return (None,) * 11
        gy = gs[0]
        d, nbytes = _desc(ctx.desc)
        L = _lib.lib()
        ws = _workspace(x.device, nbytes)
        gx = torch.empty_like(x, memory_format=_CL)
        gr = torch.empty_like(x, memory_format=_CL) if ctx.has_res else None
        gw = torch.empty_like(weight)
        gb = torch.empty_like(weight)
        bwd, name = (L.md2_bn_bwd_mask, "md2_bn_bwd_mask") if mask is not None else \
            (L.md2_bn_bwd_multi, "md2_bn_bwd_multi")
        rc = bwd(ctypes.byref(d), x.data_ptr(), mask.data_ptr() if mask is not None else None,
                 gy.data_ptr(), gs[1].data_ptr() if len(gs) > 1 else None,
                 gs[2].data_ptr() if len(gs) > 2 else None,
                 weight.data_ptr(), mean.data_ptr(), invstd.data_ptr(), gx.data_ptr(),
                 gr.data_ptr() if gr is not None else None, gw.data_ptr(), gb.data_ptr(), ws.data_ptr(),
                 _lib.stream(x.device))
        _lib.check(rc, name)
        return gx, gw, gb, None, None, gr, None, None, None, None, None


def bn_act(bn: nn.BatchNorm2d, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
           relu: bool = True, aliases: int = 0):
    """relu(bn(x) + residual) (ReLU / residual optional) for a training-mode BatchNorm2d
    (per chunk inside bn_groups).  aliases = k > 0: returns (y, y_1, ..., y_k), views of
    y for its other consumers, whose gradients the fused backward sums on load (k <= 2);
    outside the fused path the y_i are y itself."""
    if not 0 <= aliases <= 2:
        raise ValueError("bn_act: at most two aliases")
    groups = _GROUPS if bn.training else 1
    if groups > 1 and x.shape[0] % groups:
        raise ValueError(f"batch {x.shape[0]} does not split into {groups} BatchNorm groups")
    if (ENABLED and bn.training and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.dim() == 4
            and bn.affine and bn.track_running_stats and bn.momentum is not None and _supported(x.shape[1])
            and x.numel() // 4 // groups < 2 ** 31   # 32-bit element-quad index per group
            and x.is_contiguous(memory_format=_CL) and x.shape[1] > 1
            and (residual is None or residual.is_contiguous(memory_format=_CL))):
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        if bn.num_batches_tracked is not None:   # nn.BatchNorm2d counts training batches
            bn.num_batches_tracked.add_(groups)
        k = aliases if torch.is_grad_enabled() else 0
        out = _BNAct.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, residual, relu, bn.eps,
                           bn.momentum, groups, k)
        if aliases and not k:   # no graph: the aliases are y itself
            return (out,) * (aliases + 1)
        return out
    y = bn(x) if groups == 1 else torch.cat([bn(xc) for xc in x.chunk(groups)], 0)
    if residual is not None:
        y = y + residual
    y = F.relu(y) if relu else y
    return (y,) * (aliases + 1) if aliases else y


_ALIAS_SUM = os.environ.get("MD2_ALIAS_SUM", "1") != "0"


class _MaxPool(torch.autograd.Function):
    """MaxPool2d(3, 2, 1) on channels_last tensors (csrc/pool.hip).  out_alias: also
    return a view of the pooled map y for its second consumer (the first block's
    identity shortcut); with_alias: also return the input itself (a view) for x's
    second consumer (the decoder skip).  Every such gradient comes into this backward
    and is summed in the pool's gather (md2_maxpool3s2_bwd_multi) instead of by
    separate adds of the two gradients.  Outputs: (y[, y'][, x'])."""

    @staticmethod
    def forward(ctx, x, with_alias: bool = False, out_alias: bool = False):
        B, C, H, W = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        d = _lib.PoolDesc(B, C, H, W, _lib.POOL_BF16 if x.dtype == torch.bfloat16 else 0, 0)
        y = torch.empty((B, C, Ho, Wo), device=x.device, dtype=x.dtype, memory_format=_CL)
        idx = torch.empty(B * Ho * Wo * C // 4, device=x.device, dtype=torch.int32)
        stream = _lib.stream(x.device)
        _lib.check(_lib.lib().md2_maxpool3s2_fwd(ctypes.byref(d), x.data_ptr(), y.data_ptr(), idx.data_ptr(), stream),
                   "md2_maxpool3s2_fwd")
        ctx.save_for_backward(idx)
        ctx.desc = (B, C, H, W, d.flags, 0)
        ctx.xshape, ctx.dtype = x.shape, x.dtype
        ctx.with_alias, ctx.out_alias = with_alias, out_alias
        if not (with_alias or out_alias):
            return y
        ctx.set_materialize_grads(False)   # an unused output brings None, not a zero tensor
        outs = (y,) + ((y.view_as(y),) if out_alias else ()) + ((x.view_as(x),) if with_alias else ())
        return outs

    @staticmethod
    def backward(ctx, gy, *rest):
        (idx,) = ctx.saved_tensors
        rest = list(rest)
        gy2 = rest.pop(0) if ctx.out_alias else None
        galias = rest.pop(0) if ctx.with_alias else None
        if gy is None:
            gy, gy2 = gy2, None
        if gy is None:   # only the input alias reached the loss: the pool adds nothing
            return (galias.to(ctx.dtype) if galias is not None else None), None, None
        gy = gy.to(ctx.dtype).contiguous(memory_format=_CL)
        if gy2 is not None:
            gy2 = gy2.to(ctx.dtype).contiguous(memory_format=_CL)
        if galias is not None:
            galias = galias.to(ctx.dtype).contiguous(memory_format=_CL)
        gx = torch.empty(ctx.xshape, device=gy.device, dtype=ctx.dtype, memory_format=_CL)
        d = _lib.PoolDesc(*ctx.desc)
        _lib.check(_lib.lib().md2_maxpool3s2_bwd_multi(ctypes.byref(d), idx.data_ptr(), gy.data_ptr(),
                                                       gy2.data_ptr() if gy2 is not None else None,
                                                       galias.data_ptr() if galias is not None else None,
                                                       gx.data_ptr(), _lib.stream(gy.device)),
                   "md2_maxpool3s2_bwd_multi")
        return gx, None, None


def _pool_ok(pool: nn.MaxPool2d, x: torch.Tensor) -> bool:
    return (ENABLED and x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16)
            and x.shape[1] % 4 == 0 and x.is_contiguous(memory_format=_CL)
            and pool.kernel_size in (3, (3, 3)) and pool.stride in (2, (2, 2)) and pool.padding in (1, (1, 1))
            and pool.dilation in (1, (1, 1)) and not pool.ceil_mode and not pool.return_indices)


def max_pool_3x3s2(pool: nn.MaxPool2d, x: torch.Tensor) -> torch.Tensor:
    """The ResNet stem pool: HIP kernels for channels_last fp32/bf16 GPU tensors."""
    if _pool_ok(pool, x):
        return _MaxPool.apply(x, False)
    return pool(x)


def max_pool_3x3s2_with_alias(pool: nn.MaxPool2d, x: torch.Tensor, out_alias: bool = False):
    """(pool(x), x') with x' a view of x for x's other consumer (the decoder skip):
    on the HIP path both gradients of x meet in the pool's backward gather.
    out_alias: (y, y', x') with y' a view of the pooled map for its second consumer
    (the first BasicBlock's identity shortcut), whose gradient meets y's there too."""
    if _pool_ok(pool, x) and torch.is_grad_enabled() and x.requires_grad:
        if out_alias and not _ALIAS_SUM:   # A/B knob MD2_ALIAS_SUM=0: autograd adds y's two gradients
            y, xa = _MaxPool.apply(x, True, False)
            return y, y, xa
        return _MaxPool.apply(x, True, out_alias)
    y = max_pool_3x3s2(pool, x)
    return (y, y, x) if out_alias else (y, x)
