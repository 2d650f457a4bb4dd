"""Micro-benchmark of the fused photometric hot path alone (fwd+bwd) at a training shape.

    python tools/hot_bench.py [--batch 12] [--height 192] [--width 640] [--src 2] [--iters 50]

Prints one JSON line: HIP-event-timed averages of the two photometric kernels and
of the whole fwd+bwd call sequence (all 9 launches), plus algorithmic GB/s.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import monodepth2_amd  # noqa: F401,E402
import torch  # noqa: E402

from monodepth2_amd import _lib  # noqa: E402
from monodepth2_amd.data import synthetic_batch, synthetic_hotpath  # noqa: E402
from monodepth2_amd.hotpath import HotPathConfig, photometric_loss  # noqa: E402
from monodepth2_amd.layers import transformation_from_parameters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=12)
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--src", type=int, default=2)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--dump", default=None, help="save one seeded step's loss and gradients here (torch.save): "
                    "bitwise A/B of builds run with MD2_LIB")
    ap.add_argument("--no-ssim", action="store_true")
    ap.add_argument("--eight-bit", action="store_true", help="colours quantised to k/255 (loader output)")
    ap.add_argument("--src8", action="store_true", help="with --eight-bit: hand the sources' 8-bit copies "
                    "in (md2_tensors.src8, as the trainer does) instead of packing them per call")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, H, W, S = a.batch, a.height, a.width, a.src
    frame_ids = [0, -1, 1, "s"][:S + 1]
    inputs = synthetic_batch(B, H, W, frame_ids, 4, seed=0, device=dev, eight_bit=a.eight_bit)
    hp = synthetic_hotpath(B, H, W, num_src=S, seed=0, pose_scale=0.02, device=dev)
    cfg = HotPathConfig(batch=B, height=H, width=W, num_src=S, no_ssim=a.no_ssim)
    disps = [d.clone().requires_grad_(True) for d in hp["disps"]]
    Ts = []
    for i, f in enumerate(frame_ids[1:]):
        if f == "s":
            Ts.append(inputs["stereo_T"])
        else:
            Ts.append(transformation_from_parameters(hp["axisangle"][i], hp["translation"][i], invert=f < 0))
    T = torch.stack(Ts).detach().requires_grad_(True)
    colors = [[inputs[("color", f, s)] if (s == 0 or f == 0) else None for f in frame_ids] for s in range(4)]
    K = [inputs[("K", s)] for s in range(4)]
    iK = [inputs[("inv_K", s)] for s in range(4)]

    src8 = inputs.get("color_src8") if (a.src8 and a.eight_bit) else None

    def step(i):
        loss, _ = photometric_loss(cfg, disps, colors, K, iK, T, seed=i, src8=src8)
        loss[4].backward()

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with _lib.KernelTimer(2 * a.iters + 4) as kt:
        e0.record()
        for i in range(a.iters):
            step(100 + i)
        e1.record()
        torch.cuda.synchronize()
    total = e0.elapsed_time(e1) / a.iters
    N = H * W
    pyr = sum(1.0 / 4 ** s for s in range(4))
    fwd_bytes = B * N * (12 * (1 + S) + 4 * pyr + 4)
    bwd_bytes = B * N * (12 * (1 + S) + 4 * pyr + 4 + 16)
    fwd, bwd = kt.fwd_ms / kt.n_fwd, kt.bwd_ms / kt.n_bwd
    print(json.dumps({"B": B, "H": H, "W": W, "S": S, "fwd_ms": round(fwd, 4), "bwd_ms": round(bwd, 4),
                      "step_ms": round(total, 4), "fwd_GBs": round(fwd_bytes / fwd / 1e6, 1),
                      "bwd_GBs": round(bwd_bytes / bwd / 1e6, 1),
                      "hot_path_img_per_s": round(B / total * 1e3, 1)}), flush=True)
    if a.dump:
        for d in disps:
            d.grad = None
        T.grad = None
        loss, _ = photometric_loss(cfg, disps, colors, K, iK, T, seed=7, src8=src8)
        loss[4].backward()
        torch.save({"loss": loss.detach().cpu(), "disps": [d.grad.cpu() for d in disps], "T": T.grad.cpu()}, a.dump)


if __name__ == "__main__":
    main()
