"""Load the golden fixtures written by tests/golden/make_golden.py."""
from __future__ import annotations

import os
from typing import Dict

import numpy as np
import torch

from monodepth2_amd.data import synthetic_batch, synthetic_hotpath

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.endswith(".npz"))


def parse_frame(f: str):
    return f if f == "s" else int(f)


class Case:
    """A captured reference run: inputs, noise, expected outputs and gradients."""

    def __init__(self, name: str):
        self.name = name
        z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
        self.z = z
        self.B, self.H, self.W, self.S = int(z["B"]), int(z["H"]), int(z["W"]), int(z["S"])
        self.frame_ids = [parse_frame(str(f)) for f in z["frame_ids"]]
        self.flags = set(str(f) for f in z["flags"])
        self.full = "disp_0" in z.files
        self.checksums_only = "grad_disp_0" not in z.files   # large cases: scalars + checksums
        self.scales = [0, 1, 2, 3]
        self.temporal = [f for f in self.frame_ids[1:] if f != "s"]
        self.posecnn = "posecnn" in self.flags   # per-scale T (trainer.py:366-375)
        if self.full:
            self._from_arrays()
        else:
            self._regenerate()

    def _from_arrays(self):
        z = self.z
        self.disps = {s: torch.from_numpy(z[f"disp_{s}"]) for s in self.scales}
        self.inputs: Dict = {}
        for s in self.scales:
            for f in self.frame_ids:
                key = f"color_{f}_{s}"
                if key in z.files:
                    self.inputs[("color", f, s)] = torch.from_numpy(z[key])
            self.inputs[("K", s)] = torch.from_numpy(z[f"K_{s}"])
            self.inputs[("inv_K", s)] = torch.from_numpy(z[f"inv_K_{s}"])
        if "stereo_T" in z.files:
            self.inputs["stereo_T"] = torch.from_numpy(z["stereo_T"])
        self.axisangle = torch.from_numpy(z["axisangle"])
        self.translation = torch.from_numpy(z["translation"])
        self.noise = {s: torch.from_numpy(z[f"noise_{i}"]) for i, s in enumerate(self.scales)
                      if f"noise_{i}" in z.files}
        self.masks = {s: torch.from_numpy(z[f"mask_{s}"]) for s in self.scales if f"mask_{s}" in z.files}

    def _regenerate(self):
        z = self.z
        seed = int(z["seed"])
        self.inputs = synthetic_batch(self.B, self.H, self.W, self.frame_ids, 4, seed=seed,
                                      eight_bit="eight_bit" in self.flags)
        hp = synthetic_hotpath(self.B, self.H, self.W, num_src=self.S, seed=seed,
                               pose_scale=float(z["pose_scale"]))
        self.disps = {s: hp["disps"][s] for s in self.scales}
        nt = len(self.temporal)
        self.masks = {}
        self.axisangle = hp["axisangle"][:nt].clone()
        self.translation = hp["translation"][:nt].clone()
        gen = torch.Generator().manual_seed(int(z["noise_seed"]))
        self.noise = {}
        for i, s in enumerate(self.scales):
            key = f"noise_shape_{i}"
            if key in z.files:
                self.noise[s] = torch.randn(*[int(v) for v in z[key]], generator=gen)

    def expected(self, key):
        return self.z[key]


def oracle_cam_T(case: Case, axis, trans, stereo_T=None, record=None):
    """The oracle's cam_T for a case: transformation_from_parameters per temporal frame
    (trainer.py:294-295), or for posecnn a callable rebuilding T from each scale's depth
    (oracle.md2_oracle.posecnn_cam_T, trainer.py:366-375).  record: a list that gets
    (frame, T) for every T built (gradients retained), in the reference's order."""
    from monodepth2_amd.layers import transformation_from_parameters as tfp
    from oracle.md2_oracle import posecnn_cam_T
    camT = {}
    for i, f in enumerate(case.temporal):
        if case.posecnn:
            def per_scale(depth, i=i, f=f):
                T = posecnn_cam_T(tfp, axis[i], trans[i], depth, f < 0)
                if record is not None and T.requires_grad:
                    T.retain_grad()
                    record.append((f, T))
                return T
            camT[f] = per_scale
        else:
            T = tfp(axis[i], trans[i], invert=(f < 0))
            if record is not None and T.requires_grad:
                T.retain_grad()
                record.append((f, T))
            camT[f] = T
    if "s" in case.frame_ids:
        camT["s"] = stereo_T if stereo_T is not None else case.inputs["stereo_T"]
    return camT
