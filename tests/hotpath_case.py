"""Shared helpers: run a golden case through the HIP hot path and through the oracle."""
from __future__ import annotations

import torch

import numpy as np

from golden_io import Case, oracle_cam_T
from monodepth2_amd.hotpath import (HotPathConfig, generate_images, photometric_loss, predictive_mask_inputs,
                                    selection_maps)
from monodepth2_amd.layers import transformation_from_parameters


def case_config(case: Case) -> HotPathConfig:
    return HotPathConfig(batch=case.B, height=case.H, width=case.W, num_src=case.S, num_scales=4,
                         no_ssim="no_ssim" in case.flags, avg_reprojection="avg_reprojection" in case.flags,
                         disable_automasking="disable_automasking" in case.flags,
                         v1_multiscale="v1_multiscale" in case.flags,
                         predictive_mask="predictive_mask" in case.flags, t_per_scale=case.posecnn)


def _grad(t):
    """a leaf's gradient as numpy; zeros for the empty pose parameters of stereo-only cases"""
    return t.grad.cpu().numpy() if t.grad is not None else np.zeros(tuple(t.shape), np.float32)


def case_operands(case: Case, device):
    frames = case.frame_ids[1:]
    colors = [[None] * (1 + case.S) for _ in range(4)]
    for s in range(4):
        colors[s][0] = case.inputs[("color", 0, s)].to(device)
        for fi, f in enumerate(frames):
            key = ("color", f, s)
            if key in case.inputs:
                colors[s][fi + 1] = case.inputs[key].to(device)
    K = [case.inputs[("K", s)].to(device) for s in range(4)]
    inv_K = [case.inputs[("inv_K", s)].to(device) for s in range(4)]
    noise = {s: n.to(device) for s, n in case.noise.items()} if case.noise else None
    return colors, K, inv_K, noise


def run_hip(case: Case, device="cuda"):
    """Forward + backward on the GPU; returns dict of numpy results."""
    cfg = case_config(case)
    colors, K, inv_K, noise = case_operands(case, device)
    disps = [case.disps[s].to(device).clone().requires_grad_(True) for s in range(4)]
    axis = case.axisangle.to(device).clone().requires_grad_(True)
    trans = case.translation.to(device).clone().requires_grad_(True)
    if case.posecnn:
        # the product's per-scale transforms (Trainer._stacked_T): mean inverse depth of
        # each scale's upsampled depth, then one md2_pose_fwd launch per scale
        from monodepth2_amd.trainer import posecnn_transforms
        st = case.inputs["stereo_T"].to(device) if "stereo_T" in case.inputs else None
        T = posecnn_transforms(disps, axis[:, :, 0], trans[:, :, 0], case.frame_ids[1:], st, case.H, case.W,
                               cfg.min_depth, cfg.max_depth, cfg.v1_multiscale)
    else:
        Ts = []
        ti = 0
        for f in case.frame_ids[1:]:
            if f == "s":
                Ts.append(case.inputs["stereo_T"].to(device))
            else:
                Ts.append(transformation_from_parameters(axis[ti], trans[ti], invert=(f < 0)))
                ti += 1
        T = torch.stack(Ts, 0)
    if T.requires_grad:   # stereo-only: T = stereo_T, a constant
        T.retain_grad()
    masks, bce = None, None
    if cfg.predictive_mask:
        masks = {s: m.to(device).clone().requires_grad_(True) for s, m in case.masks.items()}
        up, bce = predictive_mask_inputs(cfg, masks)
        loss, sel = photometric_loss(cfg, disps, colors, K, inv_K, T, noise=noise, mask=up)
        loss = loss + torch.cat([bce, bce.mean().view(1)])   # losses["loss/s"] += BCE_s; total += mean
    else:
        loss, sel = photometric_loss(cfg, disps, colors, K, inv_K, T, noise=noise)
    loss[cfg.num_scales].backward()
    torch.cuda.synchronize()
    out = {"loss": loss.detach().cpu().numpy(), "grad_disp": [d.grad.cpu().numpy() for d in disps],
           "grad_axis": _grad(axis), "grad_trans": _grad(trans),
           "grad_T": _grad(T), "select": {s: v.cpu().numpy() for s, v in selection_maps(cfg, sel).items()}}
    if masks is not None:
        out["grad_mask"] = {s: m.grad.cpu().numpy() for s, m in masks.items()}
    with torch.no_grad():
        T2 = T.detach()
        out["gen"] = generate_images(cfg, [d.detach() for d in disps], colors, K, inv_K, T2)
    return cfg, out


def run_oracle(case: Case, selection=None, device="cpu", dtype=torch.float32):
    """The CPU oracle on the case's inputs; selection optionally pins the argmin.

    device="cuda" runs the same ATen formulation on PyTorch-ROCm (the reference's own
    ops on the GPU): a yardstick for how far two fp32 platforms of the reference
    itself drift apart at bilinear cell boundaries, never a product path.
    dtype=torch.float64: the same formulation in double precision on the same fp32
    input values — the exact-arithmetic anchor the fp32 implementations are measured
    against (pinned to the reference's own fp64 run by make_golden.py --fp64)."""
    from oracle.md2_oracle import HotPathOptions, hot_path
    opt = HotPathOptions(height=case.H, width=case.W, frame_ids=case.frame_ids,
                         v1_multiscale="v1_multiscale" in case.flags, no_ssim="no_ssim" in case.flags,
                         avg_reprojection="avg_reprojection" in case.flags,
                         disable_automasking="disable_automasking" in case.flags,
                         predictive_mask="predictive_mask" in case.flags)
    dev = torch.device(device)
    masks = ({s: m.to(dev, dtype).clone().requires_grad_(True) for s, m in case.masks.items()}
             if case.masks else None)
    disps = {s: d.to(dev, dtype).clone().requires_grad_(True) for s, d in case.disps.items()}
    axis = case.axisangle.to(dev, dtype).clone().requires_grad_(True)
    trans = case.translation.to(dev, dtype).clone().requires_grad_(True)
    inputs = {k: (v.to(dev, dtype) if torch.is_tensor(v) and v.is_floating_point() else v)
              for k, v in case.inputs.items()}
    built = []
    camT = oracle_cam_T(case, axis, trans, stereo_T=inputs.get("stereo_T"), record=built)
    sel = None
    if selection is not None:
        sel = {s: torch.from_numpy(v).long().to(dev) for s, v in selection.items()}
    noise = {s: n.to(dev, dtype) for s, n in case.noise.items()} if case.noise else None
    losses, outputs = hot_path(opt, disps, inputs, camT, noise=noise, selection=sel, masks=masks)
    losses["loss"].backward()
    res = {"loss": [float(losses[f"loss/{s}"]) for s in range(4)] + [float(losses["loss"])],
           "grad_disp": [disps[s].grad.cpu().numpy() for s in range(4)],
           "grad_axis": _grad(axis), "grad_trans": _grad(trans), "outputs": outputs}
    if case.posecnn:   # dL/dT of every per-scale T, scale-major (trainer.py:374)
        res["T"] = [T.grad.cpu().numpy() for _, T in built]
    if masks:
        res["grad_mask"] = {s: m.grad.cpu().numpy() for s, m in masks.items()}
    return res
