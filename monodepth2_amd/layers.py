"""Module-level layer API of the reference (`layers.py`), restated.

Two groups live here:

1. Building blocks that stay PyTorch-ROCm by design:
   the pose producer `transformation_from_parameters` / `rot_from_axisangle` /
   `get_translation_matrix` (tiny B x 4 x 4 work, launch-bound), and the decoder
   blocks `Conv3x3`, `ConvBlock`, `upsample` (MIOpen convolutions).
2. The per-op hot-path classes `BackprojectDepth`, `Project3D`, `SSIM`,
   `get_smooth_loss`, `disp_to_depth`, kept importable with the reference's
   constructor / forward signatures so that code written against `layers.py`
   keeps working.  They are the *unfused* eager formulation; the training hot path
   does not call them — `monodepth2_amd.hotpath` runs the whole
   warp + SSIM/L1 + min-reprojection + smoothness pipeline as fused HIP kernels.

Citations are to /root/reference/layers.py.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def disp_to_depth(disp, min_depth, max_depth):
    """Sigmoid disparity -> (scaled_disp, depth) (layers.py:16-25)."""
    lo, hi = 1.0 / max_depth, 1.0 / min_depth
    scaled = lo + (hi - lo) * disp
    return scaled, 1.0 / scaled


def rot_from_axisangle(vec: torch.Tensor) -> torch.Tensor:
    """(B,1,3) axis-angle -> (B,4,4) homogeneous rotation (layers.py:64-103).

    Rodrigues' formula with the reference's 1e-7 guard on the axis norm.
    """
    angle = torch.norm(vec, 2, 2, True)                # (B,1,1)
    axis = vec / (angle + 1e-7)
    cos, sin = torch.cos(angle), torch.sin(angle)
    one_m_cos = 1 - cos
    ax, ay, az = (axis[..., i].unsqueeze(1) for i in range(3))   # each (B,1,1)
    rows = [
        [ax * (ax * one_m_cos) + cos, ax * (ay * one_m_cos) - az * sin, az * (ax * one_m_cos) + ay * sin],
        [ax * (ay * one_m_cos) + az * sin, ay * (ay * one_m_cos) + cos, ay * (az * one_m_cos) - ax * sin],
        [az * (ax * one_m_cos) - ay * sin, ay * (az * one_m_cos) + ax * sin, az * (az * one_m_cos) + cos],
    ]
    B = vec.shape[0]
    rot = torch.zeros((B, 4, 4), device=vec.device, dtype=vec.dtype)
    for i in range(3):
        for j in range(3):
            rot[:, i, j] = rows[i][j].reshape(B)
    rot[:, 3, 3] = 1
    return rot


def get_translation_matrix(translation_vector: torch.Tensor) -> torch.Tensor:
    """(B,3) or (B,1,3) translation -> (B,4,4) (layers.py:48-61)."""
    B = translation_vector.shape[0]
    T = torch.eye(4, device=translation_vector.device,
                  dtype=translation_vector.dtype).unsqueeze(0).repeat(B, 1, 1)
    T[:, :3, 3] = translation_vector.contiguous().view(B, 3)
    return T


def transformation_from_parameters(axisangle, translation, invert=False):
    """Pose-decoder output -> 4x4 cam_T_cam (layers.py:28-45)."""
    R = rot_from_axisangle(axisangle)
    t = translation.clone()
    if invert:
        R = R.transpose(1, 2)
        t = t * -1
    T = get_translation_matrix(t)
    return torch.matmul(R, T) if invert else torch.matmul(T, R)


class Conv3x3(nn.Module):
    """Reflection- (or zero-) padded 3x3 convolution (layers.py:121-136)."""

    def __init__(self, in_channels, out_channels, use_refl=True):
        super().__init__()
        self.pad = nn.ReflectionPad2d(1) if use_refl else nn.ZeroPad2d(1)
        self.conv = nn.Conv2d(int(in_channels), int(out_channels), 3)

    def forward(self, x):
        return self.conv(self.pad(x))


class ConvBlock(nn.Module):
    """Conv3x3 followed by ELU (layers.py:106-118)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = Conv3x3(in_channels, out_channels)
        self.nonlin = nn.ELU(inplace=True)

    def forward(self, x):
        return self.nonlin(self.conv(x))


def upsample(x):
    """Nearest-neighbour x2 upsampling (layers.py:196-199)."""
    return F.interpolate(x, scale_factor=2, mode="nearest")


class BackprojectDepth(nn.Module):
    """Depth image -> homogeneous camera points (layers.py:139-168).

    Same constructor/forward signature as the reference; the pixel grid buffer is
    sized to ``batch_size`` like the reference's non-trainable parameters.
    """

    def __init__(self, batch_size, height, width):
        super().__init__()
        self.batch_size, self.height, self.width = batch_size, height, width
        ys, xs = torch.meshgrid(torch.arange(height, dtype=torch.float32),
                                torch.arange(width, dtype=torch.float32), indexing="ij")
        pix = torch.stack([xs.reshape(-1), ys.reshape(-1), torch.ones(height * width)], 0)
        self.pix_coords = nn.Parameter(pix.unsqueeze(0).repeat(batch_size, 1, 1),
                                       requires_grad=False)
        self.ones = nn.Parameter(torch.ones(batch_size, 1, height * width), requires_grad=False)

    def forward(self, depth, inv_K):
        rays = torch.matmul(inv_K[:, :3, :3], self.pix_coords)
        pts = depth.view(self.batch_size, 1, -1) * rays
        return torch.cat([pts, self.ones], 1)


class Project3D(nn.Module):
    """Camera points -> grid_sample coordinates in [-1,1] (layers.py:171-193)."""

    def __init__(self, batch_size, height, width, eps=1e-7):
        super().__init__()
        self.batch_size, self.height, self.width, self.eps = batch_size, height, width, eps

    def forward(self, points, K, T):
        P = torch.matmul(K, T)[:, :3, :]
        cam = torch.matmul(P, points)
        pix = cam[:, :2, :] / (cam[:, 2, :].unsqueeze(1) + self.eps)
        pix = pix.view(self.batch_size, 2, self.height, self.width).permute(0, 2, 3, 1)
        scale = pix.new_tensor([self.width - 1, self.height - 1])
        return (pix / scale - 0.5) * 2


def get_smooth_loss(disp, img):
    """Edge-aware first-order disparity smoothness (layers.py:202-215)."""
    ddx = (disp[:, :, :, :-1] - disp[:, :, :, 1:]).abs()
    ddy = (disp[:, :, :-1, :] - disp[:, :, 1:, :]).abs()
    idx = (img[:, :, :, :-1] - img[:, :, :, 1:]).abs().mean(1, keepdim=True)
    idy = (img[:, :, :-1, :] - img[:, :, 1:, :]).abs().mean(1, keepdim=True)
    return (ddx * torch.exp(-idx)).mean() + (ddy * torch.exp(-idy)).mean()


class SSIM(nn.Module):
    """3x3 SSIM dissimilarity with reflection padding (layers.py:218-248)."""

    C1 = 0.01 ** 2
    C2 = 0.03 ** 2

    def __init__(self):
        super().__init__()
        self.pool = nn.AvgPool2d(3, 1)
        self.refl = nn.ReflectionPad2d(1)

    def forward(self, x, y):
        x, y = self.refl(x), self.refl(y)
        mx, my = self.pool(x), self.pool(y)
        sx = self.pool(x * x) - mx * mx
        sy = self.pool(y * y) - my * my
        sxy = self.pool(x * y) - mx * my
        num = (2 * mx * my + self.C1) * (2 * sxy + self.C2)
        den = (mx * mx + my * my + self.C1) * (sx + sy + self.C2)
        return torch.clamp((1 - num / den) / 2, 0, 1)


def compute_depth_errors(gt, pred):
    """Eigen depth metrics (layers.py:251-269)."""
    ratio = torch.max(gt / pred, pred / gt)
    a1 = (ratio < 1.25).float().mean()
    a2 = (ratio < 1.25 ** 2).float().mean()
    a3 = (ratio < 1.25 ** 3).float().mean()
    rmse = torch.sqrt(((gt - pred) ** 2).mean())
    rmse_log = torch.sqrt(((torch.log(gt) - torch.log(pred)) ** 2).mean())
    abs_rel = torch.mean(torch.abs(gt - pred) / gt)
    sq_rel = torch.mean((gt - pred) ** 2 / gt)
    return abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3
