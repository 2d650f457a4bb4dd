"""ORACLE — test infrastructure only.  CPU restatement of the reference's input pipeline
(datasets/mono_dataset.py:90-200 + kitti_dataset.py:58-63) for the GPU augmentation
kernels (monodepth2_amd/csrc/augment.hip).

The reference's pixel arithmetic is PIL's (torchvision 0.2.1 transforms on PIL
images), so this module restates Pillow's integer/float algorithms exactly and is
itself pinned bit-exactly to the installed Pillow (tests/test_augment_oracle.py):

* Resize((h,w), ANTIALIAS) -> Pillow's two-pass LANCZOS resampler: coefficients
  from sinc(x)*sinc(x/3) over support 3*scale, normalised, converted to 22-bit fixed
  point, horizontal pass then vertical pass, uint8 between passes and after.
* ColorJitter (torchvision 0.2.1 get_params: b,c,s ~ U(0.8,1.2), h ~ U(-0.1,0.1),
  random order) -> ImageEnhance Brightness / Contrast / Color (Image.blend in C
  float, truncated to uint8) and adjust_hue (RGB->HSV, uint8 hue shift with
  wrap-around, HSV->RGB).  `np.uint8(hue_factor * 255)` for a negative factor wraps
  on the numpy 1.x of the reference's stack (README pins torch 0.4.1 / torchvision
  0.2.1); numpy 2 raises instead.  We restate the 1.x behaviour: trunc, mod 256.
* to_tensor: float32(u8) / 255.

`pil_*` helpers call Pillow itself and are only used to pin this restatement.
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

import numpy as np

PRECISION_BITS = 32 - 8 - 2
LANCZOS_SUPPORT = 3.0


def _sinc(x: float) -> float:
    if x == 0.0:
        return 1.0
    x = x * math.pi
    return math.sin(x) / x


def _lanczos(x: float) -> float:
    if -3.0 <= x < 3.0:
        return _sinc(x) * _sinc(x / 3.0)
    return 0.0


def lanczos_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray]:
    """Pillow precompute_coeffs + normalize_coeffs_8bpc: bounds (out,2) [xmin, n] and
    fixed-point weights (out, ksize) int32."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = LANCZOS_SUPPORT * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_lanczos((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else int(0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _resample_axis(img: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One Pillow 8-bpc pass along `axis` (0 rows, 1 columns) of an (H,W,3) uint8 image."""
    src = img.astype(np.int64)
    out_n = bounds.shape[0]
    shape = list(img.shape)
    shape[axis] = out_n
    acc = np.full(shape, 1 << (PRECISION_BITS - 1), np.int64)
    for o in range(out_n):
        xmin, n = int(bounds[o, 0]), int(bounds[o, 1])
        for x in range(n):
            if axis == 1:
                acc[:, o, :] += src[:, xmin + x, :] * int(kk[o, x])
            else:
                acc[o, :, :] += src[xmin + x, :, :] * int(kk[o, x])
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_lanczos(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """Pillow Image.resize((out_w, out_h), LANCZOS) on an (H,W,3) uint8 image."""
    h, w = img.shape[:2]
    if w != out_w:
        b, k = lanczos_coeffs(w, out_w)
        img = _resample_axis(img, b, k, axis=1)
    if h != out_h:
        b, k = lanczos_coeffs(h, out_h)
        img = _resample_axis(img, b, k, axis=0)
    return img


def to_gray(img: np.ndarray) -> np.ndarray:
    """Pillow RGB -> L: (R*19595 + G*38470 + B*7471 + 0x8000) >> 16."""
    i = img.astype(np.int64)
    return ((i[..., 0] * 19595 + i[..., 1] * 38470 + i[..., 2] * 7471 + 0x8000) >> 16).astype(np.uint8)


def blend(deg: np.ndarray, img: np.ndarray, alpha: float) -> np.ndarray:
    """Pillow ImagingBlend in C float: in1 + alpha*(in2 - in1), truncated (clipped
    when extrapolating)."""
    a = np.float32(alpha)
    if a == 0.0:
        return deg.copy()
    if a == 1.0:
        return img.copy()
    v = deg.astype(np.float32) + a * (img.astype(np.int32) - deg.astype(np.int32)).astype(np.float32)
    if 0.0 <= alpha <= 1.0:
        return v.astype(np.int32).astype(np.uint8)
    return np.where(v <= 0, 0, np.where(v >= 255, 255, v)).astype(np.int32).astype(np.uint8)


def brightness(img, f):
    return blend(np.zeros_like(img), img, f)


def contrast(img, f):
    mean = int(float(to_gray(img).astype(np.float64).mean()) + 0.5)
    return blend(np.full_like(img, mean), img, f)


def saturation(img, f):
    g = to_gray(img)
    return blend(np.repeat(g[..., None], 3, -1), img, f)


def rgb_to_hsv(img: np.ndarray) -> np.ndarray:
    """Pillow rgb2hsv_row (Convert.c), float/double as in C."""
    r, g, b = (img[..., i].astype(np.int32) for i in range(3))
    maxc = np.maximum(r, np.maximum(g, b))
    minc = np.minimum(r, np.minimum(g, b))
    cr = (maxc - minc).astype(np.float32)
    same = maxc == minc
    with np.errstate(divide="ignore", invalid="ignore"):
        s = (cr / maxc.astype(np.float32)).astype(np.float32)
        rc = ((maxc - r).astype(np.float32) / cr).astype(np.float32)
        gc = ((maxc - g).astype(np.float32) / cr).astype(np.float32)
        bc = ((maxc - b).astype(np.float32) / cr).astype(np.float32)
    h = np.where(r == maxc, (bc.astype(np.float64) - gc).astype(np.float32),
                 np.where(g == maxc, (2.0 + rc.astype(np.float64) - bc).astype(np.float32),
                          (4.0 + gc.astype(np.float64) - rc).astype(np.float32)))
    h = np.fmod(h.astype(np.float64) / 6.0 + 1.0, 1.0).astype(np.float32)
    h = np.where(same, np.float32(0), h)
    s = np.where(same, np.float32(0), s)
    uh = np.clip((h.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    us = np.clip((s.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    return np.stack([uh, us, maxc], -1).astype(np.uint8)


def _round_half_away(x: np.ndarray) -> np.ndarray:
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def hsv_to_rgb(hsv: np.ndarray) -> np.ndarray:
    """Pillow hsv2rgb (Convert.c), float/double as in C."""
    h, s, v = (hsv[..., i].astype(np.int32) for i in range(3))
    hf = h.astype(np.float32).astype(np.float64) * 6.0 / 255.0
    i = np.floor(hf).astype(np.int64)
    f = (hf - i.astype(np.float32)).astype(np.float32)
    fs = (s.astype(np.float32).astype(np.float64) / 255.0).astype(np.float32)
    vf = v.astype(np.float32).astype(np.float64)
    fs64, f64 = fs.astype(np.float64), f.astype(np.float64)
    p = np.clip(_round_half_away(vf * (1.0 - fs64)), 0, 255).astype(np.int64)
    q = np.clip(_round_half_away(vf * (1.0 - fs64 * f64)), 0, 255).astype(np.int64)
    t = np.clip(_round_half_away(vf * (1.0 - fs64 * (1.0 - f64))), 0, 255).astype(np.int64)
    i6 = i % 6
    v64 = v.astype(np.int64)
    r = np.select([i6 == 0, i6 == 1, i6 == 2, i6 == 3, i6 == 4], [v64, q, p, p, t], v64)
    g = np.select([i6 == 0, i6 == 1, i6 == 2, i6 == 3, i6 == 4], [t, v64, v64, q, p], p)
    b = np.select([i6 == 0, i6 == 1, i6 == 2, i6 == 3, i6 == 4], [p, p, t, v64, v64], q)
    out = np.stack([r, g, b], -1)
    grey = (s == 0)[..., None]
    return np.where(grey, np.repeat(v64[..., None], 3, -1), out).astype(np.uint8)


def hue_shift_u8(hue_factor: float) -> int:
    """np.uint8(hue_factor * 255) on numpy 1.x: truncate toward zero, wrap mod 256."""
    return int(math.trunc(hue_factor * 255)) % 256


def hue(img, hf):
    hsv = rgb_to_hsv(img)
    hsv[..., 0] = (hsv[..., 0].astype(np.int32) + hue_shift_u8(hf)) % 256
    return hsv_to_rgb(hsv)


def color_jitter(img: np.ndarray, order: Sequence[int], b: float, c: float, s: float, h: float) -> np.ndarray:
    """torchvision 0.2.1 ColorJitter transform built by get_params: the four adjust_*
    ops (0 brightness, 1 contrast, 2 saturation, 3 hue) applied in `order`."""
    ops = {0: lambda x: brightness(x, b), 1: lambda x: contrast(x, c), 2: lambda x: saturation(x, s),
           3: lambda x: hue(x, h)}
    for o in order:
        img = ops[int(o)](img)
    return img


def preprocess(frames: np.ndarray, height: int, width: int, num_scales: int, flip: bool, jitter):
    """mono_dataset.preprocess for one image: flip, cascaded resize, to_tensor, colour aug.
    frames: (H,W,3) uint8 native.  jitter: None or (order, b, c, s, h).
    Returns (color[s] float32 (3,h,w), color_aug[s] float32)."""
    img = frames[:, ::-1] if flip else frames
    img = np.ascontiguousarray(img)
    color, color_aug = [], []
    for s in range(num_scales):
        img = resize_lanczos(img, height // 2 ** s, width // 2 ** s)
        color.append(img.transpose(2, 0, 1).astype(np.float32) / np.float32(255))
        aug = color_jitter(img, *jitter) if jitter is not None else img
        color_aug.append(aug.transpose(2, 0, 1).astype(np.float32) / np.float32(255))
    return color, color_aug


# --- the real thing, for pinning only -------------------------------------------------
def pil_resize(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    from PIL import Image
    return np.asarray(Image.fromarray(img).resize((out_w, out_h), Image.Resampling.LANCZOS))


def pil_jitter(img: np.ndarray, order, b, c, s, h) -> np.ndarray:
    """torchvision 0.2.1 adjust_* functions written against Pillow (torchvision is not
    installed here; these are its PIL code paths)."""
    from PIL import Image, ImageEnhance
    pim = Image.fromarray(img)
    for o in order:
        if o == 0:
            pim = ImageEnhance.Brightness(pim).enhance(b)
        elif o == 1:
            pim = ImageEnhance.Contrast(pim).enhance(c)
        elif o == 2:
            pim = ImageEnhance.Color(pim).enhance(s)
        else:
            hh, ss, vv = pim.convert("HSV").split()
            np_h = np.array(hh, dtype=np.uint8)
            np_h = ((np_h.astype(np.int32) + hue_shift_u8(h)) % 256).astype(np.uint8)
            pim = Image.merge("HSV", (Image.fromarray(np_h, "L"), ss, vv)).convert("RGB")
    return np.asarray(pim)
