"""Times the GPU input pipeline (md2_aug_run) on one KITTI training batch —
F frames x B items decoded at 375x1242 -> flip + 4-level LANCZOS pyramid + jitter +
to_tensor at 192x640 — against the same work done by Pillow on the host (the
reference's DataLoader path, per-item as mono_dataset.preprocess does it).

    python tools/aug_bench.py [--batch 12] [--iters 50] [--cpu-items 4]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from monodepth2_amd.augment import GpuAugment, draw_item  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=12)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cpu-items", type=int, default=4)
    a = ap.parse_args()
    F, B, H, W, Hn, Wn = a.frames, a.batch, 192, 640, 375, 1242
    rng = np.random.default_rng(0)
    frames_np = rng.integers(0, 256, (F, B, Hn, Wn, 3), dtype=np.uint8)
    frames = torch.from_numpy(frames_np).cuda()
    r = random.Random(0)
    draws = [draw_item(r) for _ in range(B)]
    aug = GpuAugment(H, W, Hn, Wn, list(range(F)), B)
    for _ in range(5):
        aug(frames, draws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        aug(frames, draws)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    # bytes: native frames read once + u8 pyramid writes/reads + float outputs (2 per level)
    out_bytes = sum(F * B * 3 * (H >> s) * (W >> s) * 4 * 2 for s in range(4))
    in_bytes = F * B * Hn * Wn * 3

    from PIL import Image, ImageEnhance   # CPU leg: Pillow itself, as the reference's loader runs it

    def pil_jitter(arr, order, b, c, s, h):
        # torchvision 0.2.1 adjust_* on PIL (not installed here): the same Pillow calls
        pim = Image.fromarray(arr)
        for o in order:
            if o == 0:
                pim = ImageEnhance.Brightness(pim).enhance(b)
            elif o == 1:
                pim = ImageEnhance.Contrast(pim).enhance(c)
            elif o == 2:
                pim = ImageEnhance.Color(pim).enhance(s)
            else:
                hh, ss, vv = pim.convert("HSV").split()
                np_h = ((np.array(hh, dtype=np.int32) + int(h * 255)) % 256).astype(np.uint8)
                pim = Image.merge("HSV", (Image.fromarray(np_h, "L"), ss, vv)).convert("RGB")
        return np.asarray(pim)
    t0 = time.perf_counter()
    for b in range(a.cpu_items):
        d = draws[b]
        for f in range(F):
            img = Image.fromarray(frames_np[f, b])
            if d.do_flip:
                img = img.transpose(Image.Transpose.FLIP_LEFT_RIGHT)
            for s in range(4):
                img = img.resize((W >> s, H >> s), Image.Resampling.LANCZOS)
                arr = np.asarray(img)
                _ = arr.transpose(2, 0, 1).astype(np.float32) / 255
                j = pil_jitter(arr, d.order, d.brightness, d.contrast, d.saturation, d.hue) if d.do_color_aug \
                    else arr
                _ = j.transpose(2, 0, 1).astype(np.float32) / 255
    cpu_item_ms = (time.perf_counter() - t0) * 1000 / a.cpu_items
    print(json.dumps({"gpu_ms_per_batch": round(ms, 4), "batch": B, "frames": F,
                      "gpu_items_per_s": round(B / ms * 1000, 1),
                      "gpu_GBps_in_plus_out": round((in_bytes + out_bytes) / ms / 1e6, 1),
                      "pil_ms_per_item_1core": round(cpu_item_ms, 2),
                      "pil_items_per_s_1core": round(1000 / cpu_item_ms, 2)}))


if __name__ == "__main__":
    main()
