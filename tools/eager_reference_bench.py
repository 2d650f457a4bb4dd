"""The reference's formulation, run eagerly in PyTorch-ROCm on the same MI355X, beside
this build's fused step ("HIP warp+SSIM kernels vs
PyTorch-ROCm grid_sample").

Same networks, weights, optimiser and synthetic batch; the eager arm swaps in the
reference's per-op path: NCHW convolutions, nn.BatchNorm2d + ReLU (no fused BN),
DepthDecoder without the fused conv inputs, the pose matrices from
`layers.transformation_from_parameters`, and generate_images_pred + compute_losses
(trainer.py:341-496) written with `monodepth2_amd.layers` (BackprojectDepth,
Project3D, F.grid_sample, SSIM, get_smooth_loss).

    python tools/eager_reference_bench.py [--batch 12] [--steps 20] [--warmup 5]
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
import torch.nn.functional as F  # noqa: E402

import monodepth2_amd.trainer as trainer_mod  # noqa: E402
from monodepth2_amd import bn_ops  # noqa: E402
from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.layers import (SSIM, BackprojectDepth, Project3D, disp_to_depth,  # noqa: E402
                                   get_smooth_loss, transformation_from_parameters)
from monodepth2_amd.options import default_options  # noqa: E402


def eager_transforms(aa, tr, invert):
    """(F,B,3) axis-angles / translations -> (F,B,4,4), one eager chain per frame."""
    return torch.stack([transformation_from_parameters(aa[i][:, None], tr[i][:, None], invert=bool(inv))
                        for i, inv in enumerate(invert)])


class EagerTrainer(trainer_mod.Trainer):
    def __init__(self, opt, device):
        super().__init__(opt, device=device)
        self.models["depth"].fused = False
        o = self.opt
        self.ssim = SSIM().to(device)
        self.backproject = BackprojectDepth(o.batch_size, o.height, o.width).to(device)
        self.project = Project3D(o.batch_size, o.height, o.width).to(device)

    def reprojection_loss(self, pred, target):
        l1 = (target - pred).abs().mean(1, True)
        return 0.85 * self.ssim(pred, target).mean(1, True) + 0.15 * l1

    def compute_losses(self, inputs, outputs):
        o = self.opt
        srcs = o.frame_ids[1:]
        total, losses = 0, {}
        for s in range(self.num_scales):
            disp = outputs[("disp", s)]
            up = F.interpolate(disp, [o.height, o.width], mode="bilinear", align_corners=False)
            _, depth = disp_to_depth(up, o.min_depth, o.max_depth)
            target = inputs[("color", 0, 0)]
            reproj, ident = [], []
            for f in srcs:
                T = inputs["stereo_T"] if f == "s" else outputs[("cam_T_cam", 0, f)]
                pix = self.project(self.backproject(depth, inputs[("inv_K", 0)]), inputs[("K", 0)], T)
                warped = F.grid_sample(inputs[("color", f, 0)], pix, padding_mode="border", align_corners=False)
                reproj.append(self.reprojection_loss(warped, target))
                ident.append(self.reprojection_loss(inputs[("color", f, 0)], target))
            ident = torch.cat(ident, 1)
            ident = ident + torch.randn(ident.shape, device=ident.device) * 0.00001
            to_opt, _ = torch.min(torch.cat([ident, torch.cat(reproj, 1)], 1), dim=1)
            loss = to_opt.mean()
            norm = disp / (disp.mean(2, True).mean(3, True) + 1e-7)
            loss = loss + o.disparity_smoothness * get_smooth_loss(norm, inputs[("color", 0, s)]) / (2 ** s)
            losses["loss/{}".format(s)] = loss
            total = total + loss
        losses["loss"] = total / self.num_scales
        return losses


def time_steps(tr, batch, steps, warmup):
    for _ in range(warmup):
        tr.train_step(batch)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        _, losses = tr.train_step(batch)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps, float(losses["loss"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=12)
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--num_layers", type=int, default=18)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    kw = dict(batch_size=a.batch, height=a.height, width=a.width, num_layers=a.num_layers, weights_init="scratch",
              log_dir="/tmp/md2_eager")
    batch = synthetic_batch(a.batch, a.height, a.width, [0, -1, 1], 4, seed=7, device=dev)
    res = {}
    for name in ("fused", "eager"):
        torch.manual_seed(0)
        if name == "eager":
            fused_pose = trainer_mod.poses_to_transforms
            trainer_mod.poses_to_transforms = eager_transforms
            bn_ops.ENABLED = False
            tr = EagerTrainer(default_options(**kw, channels_last=0), dev)
        else:
            tr = trainer_mod.Trainer(default_options(**kw), device=dev)
        tr.set_train()
        dt, loss = time_steps(tr, batch, a.steps, a.warmup)
        if name == "eager":
            trainer_mod.poses_to_transforms = fused_pose
            bn_ops.ENABLED = True
        res[name] = {"ms_per_step": round(dt * 1e3, 3), "images_per_s": round(a.batch / dt, 2),
                     "final_loss": round(loss, 6)}
        del tr
        torch.cuda.empty_cache()
    res["speedup_fused_over_eager"] = round(res["eager"]["ms_per_step"] / res["fused"]["ms_per_step"], 3)
    res["config"] = f"mono {a.width}x{a.height} R{a.num_layers} B={a.batch} fp32, 1x MI355X"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
