"""Fused pose producer: cam_T_cam for every source frame of a step in one HIP launch.

`poses_to_transforms(axisangle (F,B,3), translation (F,B,3), invert [F]) -> (F,B,4,4)`
computes `transformation_from_parameters` (layers.py:28-45) for all frames at once
(md2_pose_fwd / md2_pose_bwd), replacing ~55 eager launches per frame each way.
On the CPU (tests, the CPU baseline) it evaluates the eager restatement in
`monodepth2_amd.layers`.
"""
from __future__ import annotations

from typing import Sequence

import torch

from . import _lib
from .layers import transformation_from_parameters


class _PoseToT(torch.autograd.Function):

    @staticmethod
    def forward(ctx, axisangle, translation, mask: int):
        aa, tr = axisangle.contiguous(), translation.contiguous()
        F_, B = aa.shape[0], aa.shape[1]
        T = torch.empty(F_, B, 4, 4, device=aa.device, dtype=aa.dtype)
        st = _lib.stream(aa.device)
        _lib.check(_lib.lib().md2_pose_fwd(F_, B, mask, aa.data_ptr(), tr.data_ptr(), T.data_ptr(), st),
                   "md2_pose_fwd")
        ctx.save_for_backward(aa, tr)
        ctx.mask = mask
        return T

    @staticmethod
    def backward(ctx, gT):
        aa, tr = ctx.saved_tensors
        gT = gT.contiguous()
        # dL/dT comes from the loss backward on the main stream; this runs on the pose
        # stream.  Mark its block in use here, or the allocator hands it back to the main
        # stream once this node has been enqueued — inside a captured step a later
        # main-stream allocation then shares its address with no order against this read
        # (C5 replays' pose-decoder bias gradients differed by a bf16 ulp, 1 run in 2)
        gT.record_stream(torch.cuda.current_stream(gT.device))
        gaa, gtr = torch.empty_like(aa), torch.empty_like(tr)
        st = _lib.stream(aa.device)
        _lib.check(_lib.lib().md2_pose_bwd(aa.shape[0], aa.shape[1], ctx.mask, aa.data_ptr(), tr.data_ptr(),
                                           gT.data_ptr(), gaa.data_ptr(), gtr.data_ptr(), st), "md2_pose_bwd")
        return gaa, gtr, None


class _Pose6ToT(torch.autograd.Function):
    """_PoseToT on one packed (F,B,6) [axisangle | translation] tensor: the gradient
    comes back as one (F,B,6) tensor (no per-slice zero-fill + copy adjoints)."""

    @staticmethod
    def forward(ctx, x6, mask: int):
        aa, tr = x6[..., :3].contiguous(), x6[..., 3:].contiguous()
        F_, B = aa.shape[0], aa.shape[1]
        T = torch.empty(F_, B, 4, 4, device=aa.device, dtype=aa.dtype)
        st = _lib.stream(aa.device)
        _lib.check(_lib.lib().md2_pose_fwd(F_, B, mask, aa.data_ptr(), tr.data_ptr(), T.data_ptr(), st),
                   "md2_pose_fwd")
        ctx.save_for_backward(aa, tr)
        ctx.mask = mask
        return T

    @staticmethod
    def backward(ctx, gT):
        aa, tr = ctx.saved_tensors
        gT = gT.contiguous()
        # dL/dT comes from the loss backward on the main stream; this runs on the pose
        # stream.  Mark its block in use here, or the allocator hands it back to the main
        # stream once this node has been enqueued — inside a captured step a later
        # main-stream allocation then shares its address with no order against this read
        # (C5 replays' pose-decoder bias gradients differed by a bf16 ulp, 1 run in 2)
        gT.record_stream(torch.cuda.current_stream(gT.device))
        gaa, gtr = torch.empty_like(aa), torch.empty_like(tr)
        st = _lib.stream(aa.device)
        _lib.check(_lib.lib().md2_pose_bwd(aa.shape[0], aa.shape[1], ctx.mask, aa.data_ptr(), tr.data_ptr(),
                                           gT.data_ptr(), gaa.data_ptr(), gtr.data_ptr(), st), "md2_pose_bwd")
        return torch.cat([gaa, gtr], -1), None


def packed_poses_to_transforms(x6: torch.Tensor, invert: Sequence[bool]) -> torch.Tensor:
    """(F,B,6) packed [axisangle | translation] (PoseDecoder.packed_output) -> (F,B,4,4)."""
    if x6.dim() != 3 or x6.shape[-1] != 6:
        raise ValueError(f"expected a (F,B,6) input, got {tuple(x6.shape)}")
    if x6.device.type != "cuda":
        return poses_to_transforms(x6[..., :3], x6[..., 3:], invert)
    if len(invert) != x6.shape[0] or len(invert) > 32:
        raise ValueError("need one invert flag per frame (at most 32 frames)")
    if x6.dtype != torch.float32:
        raise ValueError("packed_poses_to_transforms supports float32")
    return _Pose6ToT.apply(x6, sum(1 << i for i, inv in enumerate(invert) if inv))


def poses_to_transforms(axisangle: torch.Tensor, translation: torch.Tensor, invert: Sequence[bool]) -> torch.Tensor:
    """(F,B,3) axis-angles + (F,B,3) translations -> (F,B,4,4) cam_T_cam."""
    if axisangle.shape != translation.shape or axisangle.dim() != 3 or axisangle.shape[-1] != 3:
        raise ValueError(f"expected (F,B,3) inputs, got {tuple(axisangle.shape)} / {tuple(translation.shape)}")
    if len(invert) != axisangle.shape[0] or len(invert) > 32:
        raise ValueError("need one invert flag per frame (at most 32 frames)")
    if axisangle.device.type != "cuda":
        return torch.stack([transformation_from_parameters(axisangle[i].unsqueeze(1), translation[i].unsqueeze(1),
                                                           invert=bool(inv)) for i, inv in enumerate(invert)])
    if axisangle.dtype != torch.float32:
        raise ValueError("poses_to_transforms supports float32")
    mask = sum(1 << i for i, inv in enumerate(invert) if inv)
    return _PoseToT.apply(axisangle, translation, mask)
