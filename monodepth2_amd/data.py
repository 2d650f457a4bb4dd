"""Synthetic KITTI-shaped training batches.

The reference feeds `Trainer.process_batch` from `datasets/mono_dataset.py:114-200`
(JPEG decode, PIL resize pyramid, colour jitter, per-scale intrinsics).  There is
no dataset offline, so this module produces tensors with the same keys, shapes and
value ranges, deterministically from a seed:

* ``("color", f, s)`` / ``("color_aug", f, s)``: (B,3,H/2^s,W/2^s) in [0,1].  Scale 0
  is a smooth texture (sum of random-phase sinusoids + a little noise); source frames
  are the same texture seen through a small horizontal/vertical shift so that the
  photometric loss behaves like a real sequence.  Scales 1-3 are 2x2 area averages,
  standing in for the reference's resize pyramid (`mono_dataset.py:90-110`).
* ``("K", s)`` / ``("inv_K", s)``: KITTI normalised intrinsics
  (`datasets/kitti_dataset.py:29-32`) scaled per scale as `mono_dataset.py:164-173`;
  ``inv_K`` is the pseudo-inverse, as there.
* ``"stereo_T"``: identity with t_x = +-0.1 (`mono_dataset.py:192-198`) when the
  frame list contains ``"s"``.

Everything is produced on the CPU with a seeded ``torch.Generator`` and then moved
to ``device``; the same seed gives bit-identical tensors on every machine that runs
this torch build.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Sequence, Tuple, Union

import numpy as np
import torch
import torch.nn.functional as F

FrameId = Union[int, str]

# datasets/kitti_dataset.py:29-32 (normalised by image size)
KITTI_K = np.array([[0.58, 0, 0.5, 0],
                    [0, 1.92, 0.5, 0],
                    [0, 0, 1, 0],
                    [0, 0, 0, 1]], dtype=np.float32)


def scaled_intrinsics(height: int, width: int, scale: int) -> Tuple[np.ndarray, np.ndarray]:
    """K and pinv(K) for pyramid level ``scale`` (mono_dataset.py:164-173)."""
    K = KITTI_K.copy()
    K[0, :] *= width // (2 ** scale)
    K[1, :] *= height // (2 ** scale)
    inv_K = np.linalg.pinv(K).astype(np.float32)
    return K, inv_K


def _texture(gen: torch.Generator, batch: int, height: int, width: int,
             shifts: Sequence[Tuple[float, float]], n_waves: int = 8,
             noise: float = 0.02) -> List[torch.Tensor]:
    """One smooth RGB texture per image, rendered once per (dx, dy) shift."""
    yy = torch.arange(height, dtype=torch.float64).view(1, 1, height, 1)
    xx = torch.arange(width, dtype=torch.float64).view(1, 1, 1, width)
    # random wave vectors (cycles per image), phases and channel mixing
    fx = torch.rand(batch, n_waves, generator=gen, dtype=torch.float64) * 12.0 + 0.5
    fy = torch.rand(batch, n_waves, generator=gen, dtype=torch.float64) * 6.0 + 0.5
    sgn = torch.where(torch.rand(batch, n_waves, generator=gen) < 0.5, -1.0, 1.0).double()
    ph = torch.rand(batch, n_waves, generator=gen, dtype=torch.float64) * 2 * math.pi
    mix = torch.rand(batch, 3, n_waves, generator=gen, dtype=torch.float64) + 0.25
    out = []
    for dx, dy in shifts:
        arg = (2 * math.pi * (fx.view(batch, n_waves, 1, 1) * (xx + dx) / width
                              + sgn.view(batch, n_waves, 1, 1) * fy.view(batch, n_waves, 1, 1)
                              * (yy + dy) / height)
               + ph.view(batch, n_waves, 1, 1))
        waves = torch.sin(arg)                                   # (B, n, H, W)
        img = torch.einsum("bcn,bnhw->bchw", mix, waves) / mix.sum(-1).view(batch, 3, 1, 1)
        img = 0.5 + 0.45 * img
        img = img + noise * torch.randn(batch, 3, height, width, generator=gen,
                                        dtype=torch.float64)
        out.append(img.clamp(0.0, 1.0).float())
    return out


def pack_rgbx(colors: Sequence[torch.Tensor]) -> torch.Tensor:
    """The photometric sources' 8-bit copies (md2_tensors.src8): (S, B, H, W) int32 RGBx
    dwords, byte c = k of channel c, from (B, 3, H, W) colours that are exactly k/255
    (what the loader's to_tensor makes of uint8 images; md2_aug_run2 writes the same
    dwords as it decodes).  Raises if a colour is not k/255."""
    out = []
    for c in colors:
        k = torch.round(c.float() * 255.0)
        # checked on the host in float64 (exact k/255 rounded once to float32): a GPU
        # float division need not be correctly rounded
        kc = k.cpu().double()
        if not torch.equal((kc / 255.0).float(), c.float().cpu()) or bool(((kc < 0) | (kc > 255)).any()):
            raise ValueError("pack_rgbx: colours must be exactly k/255, k in 0..255")
        k = k.to(torch.int32)
        out.append(k[:, 0] | (k[:, 1] << 8) | (k[:, 2] << 16))
    return torch.stack(out).contiguous()


def synthetic_batch(batch_size: int, height: int, width: int,
                    frame_ids: Sequence[FrameId] = (0, -1, 1), num_scales: int = 4,
                    seed: int = 0, device: Union[str, torch.device] = "cpu",
                    side_sign: float = 1.0, eight_bit: bool = False) -> Dict:
    """A reference-keyed input dict for `Trainer.process_batch` (trainer.py:228).

    eight_bit: colours quantised to k/255 at every scale, as the reference's loader
    delivers them (uint8 PIL images through to_tensor, datasets/mono_dataset.py:
    199-200: float32 k / 255), plus "color_src8" — the sources' 8-bit copies
    (pack_rgbx) the hot path reads instead of packing them per step; default off to
    keep the committed fixtures' inputs.
    """
    gen = torch.Generator().manual_seed(int(seed))
    shifts = []
    for f in frame_ids:
        if f == "s":
            shifts.append((3.0 * side_sign, 0.0))           # stereo: horizontal baseline
        else:
            shifts.append((2.5 * float(f), 0.6 * float(f)))  # temporal neighbours
    imgs = _texture(gen, batch_size, height, width, shifts)
    inputs: Dict = {}
    for f, img in zip(frame_ids, imgs):
        cur = img
        for s in range(num_scales):
            if s > 0:
                cur = F.avg_pool2d(cur, 2)
            level = torch.round(cur * 255.0) / 255.0 if eight_bit else cur
            inputs[("color", f, s)] = level
            inputs[("color_aug", f, s)] = level
    if eight_bit and len(frame_ids) > 1:
        inputs["color_src8"] = pack_rgbx([inputs[("color", f, 0)] for f in frame_ids[1:]])
    for s in range(num_scales):
        K, inv_K = scaled_intrinsics(height, width, s)
        inputs[("K", s)] = torch.from_numpy(K).unsqueeze(0).repeat(batch_size, 1, 1)
        inputs[("inv_K", s)] = torch.from_numpy(inv_K).unsqueeze(0).repeat(batch_size, 1, 1)
    if "s" in frame_ids:
        T = torch.eye(4).unsqueeze(0).repeat(batch_size, 1, 1)
        T[:, 0, 3] = side_sign * 0.1
        inputs["stereo_T"] = T
    return {k: v.to(device) for k, v in inputs.items()}


def synthetic_hotpath(batch_size: int, height: int, width: int, num_src: int = 2,
                      num_scales: int = 4, seed: int = 0, pose_scale: float = 0.01,
                      device: Union[str, torch.device] = "cpu") -> Dict:
    """Decoder-shaped hot-path operands: disparities and pose parameters.

    disp_s = sigmoid(smooth field) at (B,1,H/2^s,W/2^s); axisangle/translation are
    ``pose_scale * N(0,1)`` with shape (B,1,3) as produced by the pose decoder
    (networks/pose_decoder.py:49-54).
    """
    gen = torch.Generator().manual_seed(int(seed) + 7919)
    disps = []
    base = torch.randn(batch_size, 1, max(height // 16, 2), max(width // 16, 2), generator=gen)
    for s in range(num_scales):
        h, w = height // 2 ** s, width // 2 ** s
        field = F.interpolate(base, size=(h, w), mode="bilinear", align_corners=False)
        field = field + 0.3 * torch.randn(batch_size, 1, h, w, generator=gen)
        disps.append(torch.sigmoid(field - 1.5).to(device))
    axisangle = (pose_scale * torch.randn(num_src, batch_size, 1, 3, generator=gen)).to(device)
    translation = (pose_scale * torch.randn(num_src, batch_size, 1, 3, generator=gen)).to(device)
    return {"disps": disps, "axisangle": axisangle, "translation": translation}


def frame_list(frame_ids: Iterable[FrameId], use_stereo: bool) -> List[FrameId]:
    """`trainer.py:51-52`: stereo appends the "s" frame."""
    ids = list(frame_ids)
    if use_stereo and "s" not in ids:
        ids.append("s")
    return ids
