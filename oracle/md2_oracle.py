"""ORACLE — test infrastructure only, never shipped, never on the product path.

CPU fp32 restatement of the monodepth2 per-iteration hot path:

    Trainer.generate_images_pred   (/root/reference/trainer.py:341-391)
    Trainer.compute_reprojection_loss (trainer.py:393-405)
    Trainer.compute_losses         (trainer.py:407-496)

built from the same ATen primitives the reference calls (F.interpolate bilinear,
bmm, F.grid_sample border/align_corners=False, reflection pad + 3x3 avg-pool SSIM,
torch.min), with the tie-break noise passed in explicitly instead of drawn inside
(`trainer.py:468-469`).  Gradients come from torch autograd on the CPU.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this module, and only as the checker / CPU baseline.

Pinning: checked against golden vectors captured by importing the reference itself
(`tests/golden/make_golden.py` -> `tests/golden/*.npz`, test
`tests/test_oracle_golden.py`).  The reference has no tests of its own,
so those captured vectors are the only pin.

Semantics notes (SURVEY §7 "hard parts"):
  * grid_sample align_corners defaults to False on the installed torch; the
    reference passes no value (trainer.py:384-387), so neither do we by default.
  * the identity losses are the same for every scale when v1_multiscale is off.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

SSIM_C1 = 0.01 ** 2
SSIM_C2 = 0.03 ** 2


@dataclass
class HotPathOptions:
    """The `opt.*` fields the hot path reads (trainer.py:43, 345-496)."""
    height: int = 192
    width: int = 640
    scales: Sequence[int] = (0, 1, 2, 3)
    frame_ids: Sequence = (0, -1, 1)
    min_depth: float = 0.1
    max_depth: float = 100.0
    disparity_smoothness: float = 1e-3
    v1_multiscale: bool = False
    no_ssim: bool = False
    avg_reprojection: bool = False
    disable_automasking: bool = False
    predictive_mask: bool = False
    align_corners: Optional[bool] = None     # None = torch default (False)


def depth_from_disp(disp, min_depth, max_depth):
    """layers.py:16-25."""
    lo, hi = 1 / max_depth, 1 / min_depth
    scaled = lo + (hi - lo) * disp
    return 1 / scaled


def cam_points(depth, inv_K):
    """layers.py:163-168: (B,1,h,w) depth -> (B,4,h*w) homogeneous points."""
    B, _, h, w = depth.shape
    dev, dt = depth.device, depth.dtype   # fp32 as the reference; fp64 for the parity floor
    ys, xs = torch.meshgrid(torch.arange(h, dtype=dt, device=dev),
                            torch.arange(w, dtype=dt, device=dev), indexing="ij")
    pix = torch.stack([xs.reshape(-1), ys.reshape(-1), torch.ones(h * w, dtype=dt, device=dev)], 0)
    pix = pix.unsqueeze(0).expand(B, 3, h * w)
    rays = torch.matmul(inv_K[:, :3, :3], pix)
    pts = depth.view(B, 1, -1) * rays
    return torch.cat([pts, torch.ones(B, 1, h * w, dtype=dt, device=dev)], 1)


def project(points, K, T, h, w, eps=1e-7):
    """layers.py:182-193: -> (B,h,w,2) normalised sampling grid."""
    B = points.shape[0]
    P = torch.matmul(K, T)[:, :3, :]
    cam = torch.matmul(P, points)
    pix = cam[:, :2, :] / (cam[:, 2, :].unsqueeze(1) + eps)
    pix = pix.view(B, 2, h, w).permute(0, 2, 3, 1)
    gx = (pix[..., 0] / (w - 1) - 0.5) * 2
    gy = (pix[..., 1] / (h - 1) - 0.5) * 2
    return torch.stack([gx, gy], -1)


def posecnn_cam_T(transform, axisangle, translation, depth, invert):
    """trainer.py:366-375 (pose_model_type "posecnn"): T rebuilt at every scale with
    the translation scaled by the mean inverse depth of that scale's depth map.
    axisangle / translation are the pose network's outputs at frame 0, (B,1,3)
    (`axisangle[:, 0]` of trainer.py:374); transform is transformation_from_parameters
    (layers.py:28-45), passed in so the oracle needs no product module."""
    inv_depth = 1 / depth
    mean_inv_depth = inv_depth.mean(3, True).mean(2, True)
    return transform(axisangle, translation * mean_inv_depth[:, 0], invert)


def ssim_map(x, y):
    """layers.py:234-248."""
    x = F.pad(x, (1, 1, 1, 1), mode="reflect")
    y = F.pad(y, (1, 1, 1, 1), mode="reflect")
    mx = F.avg_pool2d(x, 3, 1)
    my = F.avg_pool2d(y, 3, 1)
    sx = F.avg_pool2d(x ** 2, 3, 1) - mx ** 2
    sy = F.avg_pool2d(y ** 2, 3, 1) - my ** 2
    sxy = F.avg_pool2d(x * y, 3, 1) - mx * my
    n = (2 * mx * my + SSIM_C1) * (2 * sxy + SSIM_C2)
    d = (mx ** 2 + my ** 2 + SSIM_C1) * (sx + sy + SSIM_C2)
    return torch.clamp((1 - n / d) / 2, 0, 1)


def reprojection_loss(pred, target, no_ssim=False):
    """trainer.py:393-405: (B,3,h,w) pair -> (B,1,h,w)."""
    l1 = torch.abs(target - pred).mean(1, True)
    if no_ssim:
        return l1
    return 0.85 * ssim_map(pred, target).mean(1, True) + 0.15 * l1


def smooth_loss(disp, img):
    """layers.py:202-215 on the mean-normalised disparity (trainer.py:486-488)."""
    mean_disp = disp.mean(2, True).mean(3, True)
    d = disp / (mean_disp + 1e-7)
    gdx = torch.abs(d[:, :, :, :-1] - d[:, :, :, 1:])
    gdy = torch.abs(d[:, :, :-1, :] - d[:, :, 1:, :])
    gix = torch.mean(torch.abs(img[:, :, :, :-1] - img[:, :, :, 1:]), 1, keepdim=True)
    giy = torch.mean(torch.abs(img[:, :, :-1, :] - img[:, :, 1:, :]), 1, keepdim=True)
    return (gdx * torch.exp(-gix)).mean() + (gdy * torch.exp(-giy)).mean()


def hot_path(opt: HotPathOptions, disps: Dict[int, torch.Tensor], inputs: Dict,
             cam_T: Dict, noise: Optional[Dict[int, torch.Tensor]] = None,
             keep_images: bool = True, selection: Optional[Dict[int, torch.Tensor]] = None,
             masks: Optional[Dict[int, torch.Tensor]] = None):
    """One forward of generate_images_pred + compute_losses.

    disps: {scale: (B,1,H/2^s,W/2^s)}; inputs: reference-keyed dict with
    ("color", f, s), ("K", s), ("inv_K", s); cam_T: {frame_id: (B,4,4)} (for "s"
    pass inputs["stereo_T"]; posecnn: a callable depth -> T evaluated per scale, see
    posecnn_cam_T); noise: {scale: unit-normal tensor shaped like the
    identity losses} (trainer.py:468-469 multiplies it by 1e-5).
    selection: test-only {scale: (B,h,w) int64} pinning the per-pixel argmin of
    trainer.py:478 to given indices, so that gradients of two fp32
    implementations can be compared where rounding flips near-tied candidates.
    masks: with opt.predictive_mask, outputs["predictive_mask"][("disp", s)] at
    the native scale (trainer.py:449).

    Returns (losses, outputs) with the reference's keys.
    """
    outputs: Dict = {}
    frames = list(opt.frame_ids)[1:]
    H, W = opt.height, opt.width
    gs_kwargs = {} if opt.align_corners is None else {"align_corners": opt.align_corners}
    # --- generate_images_pred (trainer.py:341-391)
    for s in opt.scales:
        disp = disps[s]
        if opt.v1_multiscale:
            src_s = s
        else:
            disp = F.interpolate(disp, [H, W], mode="bilinear", align_corners=False)
            src_s = 0
        depth = depth_from_disp(disp, opt.min_depth, opt.max_depth)
        outputs[("depth", 0, s)] = depth
        h, w = depth.shape[2], depth.shape[3]
        for f in frames:
            T = cam_T[f](depth) if callable(cam_T[f]) else cam_T[f]
            pts = cam_points(depth, inputs[("inv_K", src_s)])
            grid = project(pts, inputs[("K", src_s)], T, h, w)
            outputs[("sample", f, s)] = grid
            outputs[("color", f, s)] = F.grid_sample(inputs[("color", f, src_s)], grid,
                                                     padding_mode="border", **gs_kwargs)
            if not opt.disable_automasking:
                outputs[("color_identity", f, s)] = inputs[("color", f, src_s)]
    # --- compute_losses (trainer.py:407-496)
    losses: Dict = {}
    total = 0
    for s in opt.scales:
        loss = 0
        src_s = s if opt.v1_multiscale else 0
        target = inputs[("color", 0, src_s)]
        reproj = torch.cat([reprojection_loss(outputs[("color", f, s)], target, opt.no_ssim)
                            for f in frames], 1)
        if not opt.disable_automasking:
            ident = torch.cat([reprojection_loss(inputs[("color", f, src_s)], target, opt.no_ssim)
                               for f in frames], 1)
            if opt.avg_reprojection:
                ident = ident.mean(1, keepdim=True)
        elif opt.predictive_mask:
            # trainer.py:447-459
            mask = masks[s]
            if not opt.v1_multiscale:
                mask = F.interpolate(mask, [H, W], mode="bilinear", align_corners=False)
            reproj = reproj * mask
            loss = loss + (0.2 * F.binary_cross_entropy(mask, torch.ones_like(mask))).mean()
        if opt.avg_reprojection:
            reproj = reproj.mean(1, keepdim=True)
        if not opt.disable_automasking:
            n = noise[s] if noise is not None else torch.randn(ident.shape)
            ident = ident + n * 0.00001
            combined = torch.cat((ident, reproj), 1)
        else:
            combined = reproj
        if combined.shape[1] == 1:
            to_opt = combined
        elif selection is not None:
            idxs = selection[s].to(torch.int64)
            to_opt = combined.gather(1, idxs.unsqueeze(1)).squeeze(1)
        else:
            to_opt, idxs = torch.min(combined, dim=1)
        if not opt.disable_automasking:
            outputs["identity_selection/{}".format(s)] = (idxs > ident.shape[1] - 1).float()
            outputs["argmin/{}".format(s)] = idxs
        loss = loss + to_opt.mean()
        loss = loss + opt.disparity_smoothness * smooth_loss(disps[s], inputs[("color", 0, s)]) / (2 ** s)
        total = total + loss
        losses["loss/{}".format(s)] = loss
    losses["loss"] = total / len(opt.scales)
    if not keep_images:
        outputs = {k: v for k, v in outputs.items() if not isinstance(k, tuple) or k[0] == "depth"}
    return losses, outputs


def noise_shapes(opt: HotPathOptions, batch: int) -> Dict[int, tuple]:
    """Shape of the tie-break noise drawn at trainer.py:468 for each scale."""
    S = len(opt.frame_ids) - 1
    ch = 1 if opt.avg_reprojection else S
    out = {}
    for s in opt.scales:
        h = opt.height // (2 ** s) if opt.v1_multiscale else opt.height
        w = opt.width // (2 ** s) if opt.v1_multiscale else opt.width
        out[s] = (batch, ch, h, w)
    return out
