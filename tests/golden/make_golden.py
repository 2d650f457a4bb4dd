"""Capture golden vectors from the reference monodepth2 hot path.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py [--ref /root/reference]

It imports the reference's own `trainer.py` / `layers.py` (stubbing the four
modules that are absent here and unused by the hot path: tensorboardX, IPython,
torchvision, skimage — SURVEY.md §8(c)), builds a minimal `self` carrying the
state `generate_images_pred` / `compute_losses` read (trainer.py:43, 145-159), and
runs the UNMODIFIED methods `Trainer.generate_images_pred` (trainer.py:341-391) and
`Trainer.compute_losses` (trainer.py:407-496) followed by `backward()`.

The tie-break noise drawn at trainer.py:468 is injected by temporarily replacing
`torch.randn` with a function that hands out pre-drawn unit-normal tensors in call
order (one per scale); the same tensors are stored in the fixture.

Poses go through the reference's `transformation_from_parameters`
(layers.py:28-45) with `invert=(f < 0)` exactly like trainer.py:294-295, so the
fixtures also pin gradients w.r.t. axisangle/translation.

Outputs: tests/golden/<case>.npz with inputs (disp_s, colours, K, inv_K,
axisangle, translation, stereo_T, noise) and outputs (loss/s, loss, warped colours,
samples, depth, identity_selection, argmin) and gradients (disp_s, axisangle,
translation, cam_T_cam).  Full-size cases store scalars and gradient checksums only.
"""
from __future__ import annotations

import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from monodepth2_amd.data import synthetic_batch, synthetic_hotpath  # noqa: E402

CASES = {
    # name: (B, H, W, frame_ids, flags, pose_scale, keep_full)
    "mono_b2_64x128": (2, 64, 128, [0, -1, 1], {}, 0.05, True),
    "stereo_b2_64x128": (2, 64, 128, [0, -1, 1, "s"], {}, 0.05, True),
    "mono_bigpose_b2_64x96": (2, 64, 96, [0, -1, 1], {}, 0.4, True),
    "no_ssim_b2_32x64": (2, 32, 64, [0, -1, 1], {"no_ssim": True}, 0.05, True),
    "avg_reproj_b2_32x64": (2, 32, 64, [0, -1, 1], {"avg_reprojection": True}, 0.05, True),
    "no_automask_b2_32x64": (2, 32, 64, [0, -1, 1], {"disable_automasking": True}, 0.05, True),
    "no_automask_avg_b2_32x64": (2, 32, 64, [0, -1, 1],
                                 {"disable_automasking": True, "avg_reprojection": True}, 0.05, True),
    "v1_multiscale_b2_64x128": (2, 64, 128, [0, -1, 1], {"v1_multiscale": True}, 0.05, True),
    "full_mono_b2_192x640": (2, 192, 640, [0, -1, 1], {}, 0.01, False),
    # the C4 resolution, and the C3 frame set (mono+stereo, S=3) at full size
    "full_mono_b2_320x1024": (2, 320, 1024, [0, -1, 1], {}, 0.01, False),
    "full_stereo_b2_192x640": (2, 192, 640, [0, -1, 1, "s"], {}, 0.01, False),
    "predictive_mask_b2_32x64": (2, 32, 64, [0, -1, 1],
                                 {"disable_automasking": True, "predictive_mask": True}, 0.05, True),
    # BASELINE configs[1] (C2): the bench's own shape, B=12 at 640x192 — losses, gradient
    # checksums and identity-selection means only (the full planes would be ~8 MB)
    # (8-bit colours, as the loader and the bench deliver them)
    "c2_mono_b12_192x640": (12, 192, 640, [0, -1, 1], {"eight_bit": True}, 0.01, False, True),
    # stereo-only training, the reference's "S" models (--use_stereo --frame_ids 0,
    # experiments/stereo_experiments.sh:2-3): one source frame, T = stereo_T, no pose net
    "stereo_only_b2_64x128": (2, 64, 128, [0, "s"], {}, 0.05, True),
    "full_stereo_only_b2_192x640": (2, 192, 640, [0, "s"], {}, 0.01, False),
    # pose_model_type posecnn: T rebuilt per scale with the translation scaled by the
    # mean inverse depth (trainer.py:366-375)
    "posecnn_b2_64x128": (2, 64, 128, [0, -1, 1], {"posecnn": True}, 0.05, True),
    "full_posecnn_b2_192x640": (2, 192, 640, [0, -1, 1], {"posecnn": True}, 0.01, False),
}


def _stub_modules():
    for name in ["tensorboardX", "IPython", "torchvision", "torchvision.models",
                 "torchvision.transforms", "skimage", "skimage.transform"]:
        if name not in sys.modules:
            m = types.ModuleType(name)
            sys.modules[name] = m
    sys.modules["tensorboardX"].SummaryWriter = object
    sys.modules["IPython"].embed = lambda *a, **k: None
    tv = sys.modules["torchvision"]
    tv.models = sys.modules["torchvision.models"]
    tv.transforms = sys.modules["torchvision.transforms"]

    class _ResNet(torch.nn.Module):       # only needed so networks/ imports
        def __init__(self, *a, **k):
            super().__init__()
    tv.models.ResNet = _ResNet
    tv.models.resnet = types.SimpleNamespace(BasicBlock=object, Bottleneck=object, model_urls={})
    for n in ["resnet18", "resnet34", "resnet50", "resnet101", "resnet152"]:
        setattr(tv.models, n, lambda *a, **k: None)


def import_reference(ref):
    _stub_modules()
    sys.path.insert(0, ref)
    import trainer as ref_trainer  # noqa: E402
    import layers as ref_layers    # noqa: E402
    return ref_trainer, ref_layers


def run_case(ref_trainer, ref_layers, name, spec, seed=0, dtype=torch.float32, pin=None):
    """dtype=torch.float64 runs the reference's methods in double precision on the same
    (fp32-valued) inputs and noise; pin = [argmin (B,h,w) per scale] then replaces the
    argmin of trainer.py:478 by the given one (the fp32 run's), so the fp64 gradients
    follow the fp32 reference's routing: the exact-arithmetic anchor (--fp64)."""
    B, H, W, frame_ids, flags, pose_scale, keep_full = spec[:7]
    checksums_only = len(spec) > 7 and spec[7]
    scales = [0, 1, 2, 3]
    S = len(frame_ids) - 1
    inputs = synthetic_batch(B, H, W, frame_ids, 4, seed=seed, eight_bit=flags.get("eight_bit", False))
    inputs = {k: (v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v) for k, v in inputs.items()}
    hp = synthetic_hotpath(B, H, W, num_src=S, seed=seed, pose_scale=pose_scale)
    disps = {s: hp["disps"][s].to(dtype).clone().requires_grad_(True) for s in scales}
    temporal = [f for f in frame_ids[1:] if f != "s"]
    axis = hp["axisangle"][:len(temporal)].to(dtype).clone().requires_grad_(True)
    trans = hp["translation"][:len(temporal)].to(dtype).clone().requires_grad_(True)

    opt = types.SimpleNamespace(
        scales=scales, frame_ids=list(frame_ids), height=H, width=W,
        v1_multiscale=flags.get("v1_multiscale", False), min_depth=0.1, max_depth=100.0,
        pose_model_type="posecnn" if flags.get("posecnn") else "separate_resnet",
        disable_automasking=flags.get("disable_automasking", False),
        no_ssim=flags.get("no_ssim", False), avg_reprojection=flags.get("avg_reprojection", False),
        predictive_mask=flags.get("predictive_mask", False), disparity_smoothness=1e-3, batch_size=B)
    self = types.SimpleNamespace(opt=opt, device=torch.device("cpu"), num_scales=len(scales))
    self.ssim = ref_layers.SSIM().to(dtype)
    self.backproject_depth, self.project_3d = {}, {}
    for s in scales:
        h, w = H // 2 ** s, W // 2 ** s
        self.backproject_depth[s] = ref_layers.BackprojectDepth(B, h, w).to(dtype)
        self.project_3d[s] = ref_layers.Project3D(B, h, w).to(dtype)
    self.compute_reprojection_loss = types.MethodType(
        ref_trainer.Trainer.compute_reprojection_loss, self)

    outputs = {("disp", s): disps[s] for s in scales}
    masks = {}
    if flags.get("predictive_mask"):
        # the mask decoder's sigmoid outputs (B, S, h_s, w_s) (trainer.py:96-98, 252)
        mgen = torch.Generator().manual_seed(seed + 777)
        for s in scales:
            h, w = H // 2 ** s, W // 2 ** s
            masks[s] = torch.sigmoid(torch.randn(B, S, h, w, generator=mgen)).requires_grad_(True)
        outputs["predictive_mask"] = {("disp", s): masks[s] for s in scales}
    # the reference builds its pose matrices from torch.zeros() (layers.py:53, 93), i.e.
    # in the default dtype: an fp64 run makes that the default from here on (the inputs
    # above and the noise draws below are fp32 values either way)
    real_default = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    camT = {}
    for i, f in enumerate(temporal):
        T = ref_layers.transformation_from_parameters(axis[i], trans[i], invert=(f < 0))
        T.retain_grad()
        outputs[("cam_T_cam", 0, f)] = T
        camT[f] = T
        if flags.get("posecnn"):
            # the pose network's (B, frames=1, 1, 3) outputs (networks/pose_cnn.py:45-50):
            # generate_images_pred reads axisangle[:, 0] / translation[:, 0]
            outputs[("axisangle", 0, f)] = axis[i].unsqueeze(1)
            outputs[("translation", 0, f)] = trans[i].unsqueeze(1)
    # posecnn: the per-scale T of trainer.py:374-375, recorded as the reference builds
    # them (scale-major, frame-minor) with their gradients
    per_scale_T = []
    real_tfp = ref_trainer.transformation_from_parameters

    def recording_tfp(*a, **k):
        T = real_tfp(*a, **k)
        T.retain_grad()
        per_scale_T.append(T)
        return T

    # noise injection (trainer.py:468)
    gen = torch.Generator().manual_seed(seed + 12345)
    drawn = []
    real_randn = torch.randn

    def fake_randn(shape, device=None, **kw):
        n = real_randn(*shape, generator=gen, dtype=torch.float32)
        drawn.append(n.clone())
        return n.to(dtype)

    # the per-pixel argmin of trainer.py:478 (torch.min(combined, dim=1)), recorded as the
    # reference computes it: the tests compare gradients away from pixels whose argmin
    # differs (an fp32 near-tie re-routes that pixel's gradient)
    argmins = []
    real_min = torch.min

    def recording_min(*a, **k):
        if not (k.get("dim") == 1 or (len(a) > 1 and a[1] == 1)):
            return real_min(*a, **k)
        if pin is not None:   # the given argmin; min's gradient routing through gather
            idx = torch.from_numpy(pin[len(argmins)].astype(np.int64))
            r = (a[0].gather(1, idx.unsqueeze(1)).squeeze(1), idx)
        else:
            r = real_min(*a, **k)
        argmins.append(r[1].clone())
        return r

    ref_trainer.torch.randn = fake_randn
    ref_trainer.torch.min = recording_min
    ref_trainer.transformation_from_parameters = recording_tfp
    real_cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda t, *a, **k: t     # trainer.py:458 calls .cuda(); CPU-only here
    try:
        ref_trainer.Trainer.generate_images_pred(self, inputs, outputs)
        losses = ref_trainer.Trainer.compute_losses(self, inputs, outputs)
    finally:
        ref_trainer.torch.randn = real_randn
        ref_trainer.torch.min = real_min
        ref_trainer.transformation_from_parameters = real_tfp
        torch.Tensor.cuda = real_cuda
    try:
        losses["loss"].backward()
    finally:
        torch.set_default_dtype(real_default)

    rec = {"B": B, "H": H, "W": W, "S": S, "seed": seed, "pose_scale": pose_scale,
           "frame_ids": np.array([str(f) for f in frame_ids]),
           "flags": np.array(sorted(k for k, v in flags.items() if v))}
    for s in scales:
        rec[f"loss_{s}"] = losses[f"loss/{s}"].detach().numpy()
        if not checksums_only:
            rec[f"grad_disp_{s}"] = disps[s].grad.numpy()
    rec["loss"] = losses["loss"].detach().numpy()
    if len(argmins) == len(scales):
        for s, idx in zip(scales, argmins):
            rec[f"argmin_{s}"] = idx.numpy().astype(np.uint8)
    if temporal:   # stereo-only: no pose parameters
        rec["grad_axisangle"] = axis.grad.numpy()
        rec["grad_translation"] = trans.grad.numpy()
    for s, m in masks.items():
        rec[f"mask_{s}"] = m.detach().numpy()
        rec[f"grad_mask_{s}"] = m.grad.numpy()
    for f in temporal:
        if camT[f].grad is not None:   # posecnn: the per-scale T below carry the gradient
            rec[f"grad_T_{f}"] = camT[f].grad.numpy()
        rec[f"T_{f}"] = camT[f].detach().numpy()
    if flags.get("posecnn"):
        assert len(per_scale_T) == len(scales) * len(temporal), len(per_scale_T)
        for j, T in enumerate(per_scale_T):
            s, f = scales[j // len(temporal)], temporal[j % len(temporal)]
            rec[f"T_{f}_{s}"] = T.detach().numpy()
            rec[f"grad_T_{f}_{s}"] = T.grad.numpy()
    if keep_full:
        for s in scales:
            rec[f"disp_{s}"] = hp["disps"][s].numpy()
            for f in frame_ids:
                if s == 0 or f == 0 or flags.get("v1_multiscale"):
                    rec[f"color_{f}_{s}"] = inputs[("color", f, s)].numpy()
            rec[f"K_{s}"] = inputs[("K", s)].numpy()
            rec[f"inv_K_{s}"] = inputs[("inv_K", s)].numpy()
            rec[f"depth_{s}"] = outputs[("depth", 0, s)].detach().numpy()
            for f in frame_ids[1:]:
                rec[f"warp_{f}_{s}"] = outputs[("color", f, s)].detach().numpy()
                rec[f"sample_{f}_{s}"] = outputs[("sample", f, s)].detach().numpy()
            if not opt.disable_automasking:
                rec[f"identity_selection_{s}"] = outputs[f"identity_selection/{s}"].numpy().astype(np.uint8)
        rec["axisangle"] = axis.detach().numpy()
        rec["translation"] = trans.detach().numpy()
        if "stereo_T" in inputs:
            rec["stereo_T"] = inputs["stereo_T"].numpy()
        for i, n in enumerate(drawn):
            rec[f"noise_{i}"] = n.numpy()
    else:
        for i, n in enumerate(drawn):
            rec[f"noise_shape_{i}"] = np.array(n.shape)
        rec["noise_seed"] = seed + 12345
        for s in scales:
            g = disps[s].grad
            rec[f"grad_disp_sum_{s}"] = g.double().sum().numpy()
            rec[f"grad_disp_abs_{s}"] = g.double().abs().sum().numpy()
            rec[f"grad_disp_sq_{s}"] = g.double().square().sum().numpy()
            # per-image abs sums: a gradient routed to the wrong image shows up here
            rec[f"grad_disp_abs_img_{s}"] = g.double().abs().sum((1, 2, 3)).numpy()
            if not opt.disable_automasking:
                rec[f"identity_selection_mean_{s}"] = outputs[f"identity_selection/{s}"].double().mean().numpy()
    return rec


# the full-size cases whose gradient parity is anchored on the fp64 floor
FP64_CASES = ["full_mono_b2_192x640", "full_mono_b2_320x1024", "full_stereo_b2_192x640", "c2_mono_b12_192x640",
              "full_stereo_only_b2_192x640", "full_posecnn_b2_192x640"]
F64_KEYS = ("loss", "loss_", "grad_disp_sum_", "grad_disp_abs_", "grad_disp_sq_", "grad_disp_abs_img_",
            "grad_axisangle", "grad_translation", "grad_T_")


def add_fp64(ref_trainer, ref_layers, name):
    """Augment an existing fixture with the reference's own fp64 run (argmin pinned to
    the fixture's fp32 argmin): scalars and gradient checksums under "f64_*" keys.
    tests/test_oracle_golden.py pins the oracle's fp64 mode to them; the GPU floor test
    then measures the HIP path and the fp32 oracle against that fp64 oracle."""
    path = os.path.join(HERE, name + ".npz")
    z = dict(np.load(path, allow_pickle=False))
    spec = CASES[name]
    spec64 = spec[:6] + (False, True)   # checksums only
    pin = [z[f"argmin_{s}"] for s in range(4)]
    rec = run_case(ref_trainer, ref_layers, name, spec64, seed=int(z["seed"]), dtype=torch.float64, pin=pin)
    for k, v in rec.items():
        if k.startswith(F64_KEYS) and not k.startswith("loss_shape"):
            z["f64_" + k] = v
    np.savez_compressed(path, **z)
    print(f"{name}: fp64 loss={float(rec['loss']):.10f} (fp32 {float(z['loss']):.7f}) -> {os.path.relpath(path, REPO)}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None)
    ap.add_argument("--fp64", action="store_true", help="add the fp64 anchors to the full-size fixtures")
    args = ap.parse_args()
    torch.set_num_threads(8)
    ref_trainer, ref_layers = import_reference(args.ref)
    if args.fp64:
        for name in FP64_CASES:
            if not args.only or name == args.only:
                add_fp64(ref_trainer, ref_layers, name)
        return
    for name, spec in CASES.items():
        if args.only and name != args.only:
            continue
        rec = run_case(ref_trainer, ref_layers, name, spec)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **rec)
        print(f"{name}: loss={float(rec['loss']):.7f} -> {os.path.relpath(path, REPO)} "
              f"({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
