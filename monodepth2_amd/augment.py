"""GPU input pipeline: the per-item work of `MonoDataset.__getitem__` for a whole batch
in HIP (csrc/augment.hip, ABI `md2_aug_*` in include/md2hot.h).

The reference (datasets/mono_dataset.py:114-200) decodes each frame, flips it
(kitti_dataset.py:58-63), builds the Resize(ANTIALIAS) pyramid by cascading from the
previous level (mono_dataset.py:80-84, 96-101), and stores ToTensor of every level
as ("color", f, s) and of ColorJitter(level) as ("color_aug", f, s), with one jitter
draw shared by all frames of an item (mono_dataset.py:175-181).  Here the decoded
uint8 frames of a batch sit in HBM and one `md2_aug_run` produces every key; the
outputs equal the reference's PIL pipeline byte for byte (tests/test_augment_gpu.py).

Random decisions stay on the host, drawn with Python's `random` in the reference's
order: do_color_aug, do_flip (mono_dataset.py:136-137), then torchvision 0.2.1
`ColorJitter.get_params(0.2, 0.2, 0.2, 0.1)` (the scalar fallback the reference
takes on that version, mono_dataset.py:66-78): brightness, contrast, saturation
~ U(0.8, 1.2), hue ~ U(-0.1, 0.1), then `random.shuffle` of the four transforms.
"""
from __future__ import annotations

import ctypes
import math
import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .data import scaled_intrinsics


@dataclass
class ItemDraw:
    """One item's random decisions (what MonoDataset.__getitem__ draws)."""
    do_color_aug: bool = False
    do_flip: bool = False
    brightness: float = 1.0
    contrast: float = 1.0
    saturation: float = 1.0
    hue: float = 0.0
    order: List[int] = field(default_factory=lambda: [0, 1, 2, 3])   # 0 b, 1 c, 2 s, 3 h


def draw_item(rng: random.Random, is_train: bool = True) -> ItemDraw:
    """The reference's draws for one item, in its order (mono_dataset.py:136-137,
    175-179 with torchvision 0.2.1 ColorJitter.get_params)."""
    d = ItemDraw()
    d.do_color_aug = is_train and rng.random() > 0.5
    d.do_flip = is_train and rng.random() > 0.5
    if d.do_color_aug:
        d.brightness = rng.uniform(0.8, 1.2)
        d.contrast = rng.uniform(0.8, 1.2)
        d.saturation = rng.uniform(0.8, 1.2)
        d.hue = rng.uniform(-0.1, 0.1)
        rng.shuffle(d.order)
    return d


def hue_shift(hue_factor: float) -> int:
    """`np.uint8(hue_factor * 255)` (torchvision 0.2.1 adjust_hue) as numpy 1.x
    evaluates it: truncation toward zero, then wrap modulo 256."""
    return int(math.trunc(hue_factor * 255)) % 256


def pack_items(draws: Sequence[ItemDraw]):
    """md2_aug_item[B] (host ctypes array; md2_aug_run stages it through pinned memory)."""
    arr = (_lib.AugItem * len(draws))()
    for a, d in zip(arr, draws):
        a.flip = int(d.do_flip)
        a.color_aug = int(d.do_color_aug)
        a.hue_shift = hue_shift(d.hue) if d.do_color_aug else 0
        for k in range(4):
            a.order[k] = d.order[k]
        a.brightness, a.contrast, a.saturation = d.brightness, d.contrast, d.saturation
    return arr


class GpuAugment:
    """Batch-level MonoDataset preprocessing on the GPU.

    frames: uint8 (F, B, in_height, in_width, 3) on the device, frame-major in the
    order of `frame_ids`.  Returns the reference's input dict: ("color", f, s),
    ("color_aug", f, s) (B,3,h_s,w_s) float32, ("K", s) / ("inv_K", s) (B,4,4) and,
    with "s" in frame_ids, "stereo_T" (B,4,4)."""

    def __init__(self, height: int, width: int, in_height: int, in_width: int, frame_ids: Sequence,
                 batch_size: int, num_scales: int = 4, device="cuda"):
        self.height, self.width = height, width
        self.in_height, self.in_width = in_height, in_width
        self.frame_ids = list(frame_ids)
        self.batch_size = batch_size
        self.num_scales = num_scales
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("GpuAugment runs on the GPU only (no CPU fallback)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        L = _lib.lib()
        desc = _lib.AugDesc(batch_size, len(self.frame_ids), in_height, in_width, height, width, num_scales, 0)
        with torch.cuda.device(self.device):
            self._plan = L.md2_aug_plan_create(ctypes.byref(desc))
        if not self._plan:
            raise RuntimeError("md2_aug_plan_create failed: " + L.md2_last_error().decode(errors="replace"))
        self._K = {}
        for s in range(num_scales):
            K, inv_K = scaled_intrinsics(height, width, s)
            rep = lambda m: torch.from_numpy(m).to(self.device).unsqueeze(0).repeat(batch_size, 1, 1)
            self._K[s] = (rep(K), rep(inv_K))

    def __del__(self):
        plan = getattr(self, "_plan", None)
        if plan:
            try:
                _lib.lib().md2_aug_plan_destroy(plan)
            except Exception:
                pass
            self._plan = None

    def run(self, frames: torch.Tensor, items):
        """Raw call (items = pack_items(...)): returns (color[s], color_aug[s]) tensors
        shaped (F,B,3,h,w)."""
        F, B = len(self.frame_ids), self.batch_size
        want = (F, B, self.in_height, self.in_width, 3)
        if tuple(frames.shape) != want or frames.dtype != torch.uint8 or not frames.is_contiguous():
            raise ValueError(f"frames must be contiguous uint8 {want}, got {tuple(frames.shape)} {frames.dtype}")
        if frames.device != self.device:
            raise ValueError("frames must live on the plan's device")
        if len(items) != B:
            raise ValueError("items must hold one md2_aug_item per batch item")
        color, color_aug = [], []
        for s in range(self.num_scales):
            shp = (F, B, 3, self.height >> s, self.width >> s)
            color.append(torch.empty(shp, device=self.device))
            color_aug.append(torch.empty(shp, device=self.device))
        cp = (ctypes.c_void_p * self.num_scales)(*[t.data_ptr() for t in color])
        ap = (ctypes.c_void_p * self.num_scales)(*[t.data_ptr() for t in color_aug])
        # the photometric sources (frames 1..F-1) at scale 0 as 8-bit RGBx dwords too
        self.src8 = torch.empty((F - 1, B, self.height, self.width), dtype=torch.int32,
                                device=self.device) if F > 1 else None
        stream = _lib.stream(self.device)
        _lib.check(_lib.lib().md2_aug_run2(self._plan, frames.data_ptr(), ctypes.byref(items), cp, ap,
                                           self.src8.data_ptr() if self.src8 is not None else None, stream),
                   "md2_aug_run2")
        return color, color_aug

    def __call__(self, frames: torch.Tensor, draws: Sequence[ItemDraw], sides: Optional[Sequence[str]] = None
                 ) -> Dict:
        color, color_aug = self.run(frames, pack_items(draws))
        inputs = {}
        for s in range(self.num_scales):
            for i, f in enumerate(self.frame_ids):
                inputs[("color", f, s)] = color[s][i]
                inputs[("color_aug", f, s)] = color_aug[s][i]
            K, inv_K = self._K[s]
            inputs[("K", s)] = K
            inputs[("inv_K", s)] = inv_K
        if self.src8 is not None:   # the hot path's 8-bit sources (md2_tensors.src8)
            inputs["color_src8"] = self.src8
        if "s" in self.frame_ids:
            # mono_dataset.py:192-198: t_x = side_sign * baseline_sign * 0.1
            # the side comes from each split line (mono_dataset.py:136-140); no default:
            # a wrong side flips the sign of the stereo baseline
            if sides is None or len(sides) != self.batch_size or any(sd not in ("l", "r") for sd in sides):
                raise ValueError("GpuAugment: stereo frame ids need one side ('l'/'r') per item, "
                                 f"got {sides!r} for batch {self.batch_size}")
            T = np.tile(np.eye(4, dtype=np.float32), (self.batch_size, 1, 1))
            for b, (d, side) in enumerate(zip(draws, sides)):
                T[b, 0, 3] = (-1 if side == "l" else 1) * (-1 if d.do_flip else 1) * 0.1
            inputs["stereo_T"] = torch.from_numpy(T).to(self.device)
        return inputs
