"""Training step with the fused HIP photometric hot path.

Counterpart of the reference `Trainer` (trainer.py:29-630) restricted to what a
training step needs.  The networks stay PyTorch-ROCm modules (networks/*);
`generate_images_pred` + `compute_losses` (trainer.py:341-496) run as ONE fused
autograd op over hand-written HIP kernels (`monodepth2_amd.hotpath`).

Differences from the reference, all deliberate:
  * data comes from an iterable of reference-keyed batches (synthetic KITTI-shaped
    tensors by default, `data.synthetic_batch`) instead of the JPEG loader;
  * the tie-break noise of trainer.py:468 is drawn inside the kernel from a
    counter-based generator (seed = noise_seed, step, rank) — no randn launches;
  * `generate_images_pred` materialises warped colours / samples / depth only when
    asked (logging, evaluation or `--materialize_images`), because the fused loss
    does not need them;
  * data parallelism: one process per GPU, DDP over RCCL (backend "nccl") with the
    gradient all-reduce bucketed and overlapped with the backward pass.  The
    reference is single-GPU (README.md:147-155).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Iterable, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim

from . import conv_ops, networks
from .distributed import FlatGradSync, wrap_ddp
from .hotpath import HotPathConfig, generate_images, photometric_loss, predictive_mask_inputs, selection_maps
from .bn_ops import bn_groups
from .layers import compute_depth_errors, disp_to_depth
from .optim import FusedAdam
from .pose_ops import packed_poses_to_transforms, poses_to_transforms


def _sec_to_hm_str(t):
    t = int(t)
    s = t % 60
    t //= 60
    m = t % 60
    t //= 60
    return "{:02d}h{:02d}m{:02d}s".format(t, m, s)


def _to_fp32(outputs, keep_disp: bool = True):
    """Network outputs (nested dicts of tensors) as fp32 (--amp bf16).  The depth
    decoder's disparities stay as they are: the fused hot path reads bf16 disparities
    directly (md2_desc.disp_dtype) and returns their gradients in bf16, which is what
    a cast up and its backward would give, without the two extra passes."""
    if isinstance(outputs, dict):
        return {k: (v if (keep_disp and isinstance(k, tuple) and len(k) == 2 and k[0] == "disp")
                    else _to_fp32(v, keep_disp=False)) for k, v in outputs.items()}
    if torch.is_tensor(outputs) and outputs.is_floating_point() and outputs.dtype != torch.float32:
        return outputs.float()
    return outputs


def posecnn_transforms(disps, axisangle, translation, src_frames, stereo_T, height: int, width: int,
                       min_depth: float, max_depth: float, v1_multiscale: bool) -> torch.Tensor:
    """pose_model_type "posecnn" (trainer.py:366-375): cam_T_cam rebuilt at every scale
    with the translation scaled by the mean inverse depth of that scale's depth map
    (upsampled to the loss resolution unless v1_multiscale).  axisangle / translation:
    (F,B,3) for the temporal source frames in frame order.  Returns the
    (num_scales, S, B, 4, 4) stack the hot path takes with t_per_scale (stereo_T for an
    "s" frame).  The mean inverse depth is formed as the reference forms it, 1 / (1 /
    scaled disparity), then the transforms of a scale come from one md2_pose_fwd launch."""
    temporal = [f for f in src_frames if f != "s"]
    per_scale = []
    for d in disps:
        d = d.float()
        if not v1_multiscale:
            d = F.interpolate(d, [height, width], mode="bilinear", align_corners=False)
        _, depth = disp_to_depth(d, min_depth, max_depth)
        mean_inv_depth = (1 / depth).mean(3, True).mean(2, True)          # (B,1,1,1)
        Tt = poses_to_transforms(axisangle, translation * mean_inv_depth[:, 0, 0].unsqueeze(0),
                                 [f < 0 for f in temporal])
        Ts, ti = [], 0
        for f in src_frames:
            if f == "s":
                Ts.append(stereo_T)
            else:
                Ts.append(Tt[ti])
                ti += 1
        per_scale.append(torch.stack(Ts, 0))
    return torch.stack(per_scale, 0)


def _check_graph_backend(hip_graph: bool, world_size: int) -> None:
    """A captured step at world size > 1 holds the gradient all-reduce inside the
    hipGraph (FlatGradSync on its communication stream), which only RCCL ("nccl") can
    enqueue under stream capture: gloo's host-side all-reduce raises
    hipErrorStreamCaptureUnsupported in the middle of the capture.  Refuse the
    combination up front, before any network is built (trainer.py:201-210 is the
    reference's single-process step this distributes)."""
    if not hip_graph or world_size <= 1:
        return
    backend = dist.get_backend() if (dist.is_available() and dist.is_initialized()) else None
    if backend != "nccl":
        raise ValueError(
            f"--hip_graph at world size {world_size} needs the RCCL process group (backend 'nccl'); "
            f"got {backend!r}: a {backend} all-reduce cannot be captured into a hipGraph.  "
            "Run the eager step (hip_graph off / bench.py --graph 0) on this backend.")


class _Networks(nn.Module):
    """All trainable networks behind one module so DDP sees a single graph."""

    def __init__(self, models: Dict[str, nn.Module]):
        super().__init__()
        self.models = nn.ModuleDict(models)

    def forward(self, trainer: "Trainer", inputs):
        return trainer._run_networks(self.models, inputs)


# diagnosis knobs (C5 graph-replay determinism): the logging maps on the main stream,
# the pose stream joined to the main one before the backward, the pose network second
_LOGMAPS_SIDE = os.environ.get("MD2_LOGMAPS_SIDE", "1") != "0"
_JOIN_BEFORE_BWD = os.environ.get("MD2_JOIN_BEFORE_BWD", "0") == "1"
_POSE_LAST = os.environ.get("MD2_POSE_LAST", "0") == "1"

class Trainer:
    def __init__(self, options, device: Optional[torch.device] = None, rank: int = 0, world_size: int = 1):
        self.opt = options
        self.log_path = os.path.join(self.opt.log_dir, self.opt.model_name)
        assert self.opt.height % 32 == 0, "'height' must be a multiple of 32"
        assert self.opt.width % 32 == 0, "'width' must be a multiple of 32"
        if self.opt.no_cuda:
            raise RuntimeError("the MI355X build has no CPU training path: the hot path is HIP-only")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.rank, self.world_size = rank, world_size
        _check_graph_backend(bool(getattr(self.opt, "hip_graph", False)), world_size)

        self.num_scales = len(self.opt.scales)
        if list(self.opt.scales) != list(range(self.num_scales)):
            raise ValueError("scales must be 0..n-1 (got {})".format(self.opt.scales))
        self.num_input_frames = len(self.opt.frame_ids)
        self.num_pose_frames = 2 if self.opt.pose_model_input == "pairs" else self.num_input_frames
        assert self.opt.frame_ids[0] == 0, "frame_ids must start with 0"
        self.use_pose_net = not (self.opt.use_stereo and self.opt.frame_ids == [0])
        if self.opt.use_stereo and "s" not in self.opt.frame_ids:
            self.opt.frame_ids = list(self.opt.frame_ids) + ["s"]
        if self.opt.predictive_mask:
            assert self.opt.disable_automasking, \
                "When using predictive_mask, please disable automasking with --disable_automasking"

        pretrained = self.opt.weights_init == "pretrained"
        self.models: Dict[str, nn.Module] = {}
        self.models["encoder"] = networks.ResnetEncoder(self.opt.num_layers, pretrained)
        self.models["depth"] = networks.DepthDecoder(self.models["encoder"].num_ch_enc, self.opt.scales)
        if self.use_pose_net:
            if self.opt.pose_model_type == "separate_resnet":
                self.models["pose_encoder"] = networks.ResnetEncoder(
                    self.opt.num_layers, pretrained, num_input_images=self.num_pose_frames)
                self.models["pose"] = networks.PoseDecoder(self.models["pose_encoder"].num_ch_enc,
                                                           num_input_features=1, num_frames_to_predict_for=2)
            elif self.opt.pose_model_type == "shared":
                self.models["pose"] = networks.PoseDecoder(self.models["encoder"].num_ch_enc, self.num_pose_frames)
            elif self.opt.pose_model_type == "posecnn":
                self.models["pose"] = networks.PoseCNN(
                    self.num_input_frames if self.opt.pose_model_input == "all" else 2)
        if self.opt.predictive_mask:
            # same architecture as the depth decoder, one mask per source frame (trainer.py:94-100)
            self.models["predictive_mask"] = networks.DepthDecoder(
                self.models["encoder"].num_ch_enc, self.opt.scales,
                num_output_channels=(len(self.opt.frame_ids) - 1))
        for m in self.models.values():
            m.to(self.device)
            if getattr(self.opt, "channels_last", False):
                m.to(memory_format=torch.channels_last)
        self.nets = _Networks(self.models)
        self.parameters_to_train = [p for m in self.models.values() for p in m.parameters()]
        # BatchNorm's num_batches_tracked only matters with momentum=None (never used
        # here or in the reference), yet costs one tiny launch per BN layer per step:
        # keep one step counter instead and write it back into checkpoints.
        # Calls per step differ: the separate pose encoder runs once per frame pair in
        # the reference (trainer.py:280-290), so its layers count that many batches.
        self._bn_layers, self._bn_mult = [], []
        pairs = sum(1 for f in self.opt.frame_ids[1:] if f != "s")
        for name, m in self.nets.named_modules():
            if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.momentum is not None \
                    and m.num_batches_tracked is not None:
                self._bn_layers.append(m)
                self._bn_mult.append(pairs if (name.startswith("models.pose_encoder.")
                                               and self.num_pose_frames == 2) else 1)
                m.num_batches_tracked = None
        self._bn_steps = 0
        self.batch_pose_pairs = True   # one pose-encoder pass over all frame pairs (bn_groups)
        # second HIP stream for the pose network (overlaps the depth network).  Under
        # hipGraph capture the fork/join (event record + wait) is captured too, so the
        # graph keeps the two branches independent.
        self._pose_stream = (torch.cuda.Stream(self.device)
                             if self.device.type == "cuda" and getattr(self.opt, "pose_streams", 1) else None)
        self._in_step = False   # inside _step_body (compute_losses' logging maps go to the pose stream)

        # gradient averaging: DDP (hooks, overlapped with backward) for eager steps, flat
        # buckets + one RCCL all-reduce each (graph-capturable) for --hip_graph
        self.use_graph = bool(getattr(self.opt, "hip_graph", False))
        if (self.use_graph and self.device.type == "cuda" and self._pose_stream is None
                and os.environ.get("MD2_ALLOW_ONESTREAM_GRAPH", "0") != "1"):
            # open bug: a captured step with the pose network on the main
            # stream replays with non-finite gradients for some parameters after one or more
            # replays (tools/onestream_graph_check.py; fp32 and bf16); the default two-stream
            # capture is bitwise the eager step.  Refused rather than trained on silently.
            raise ValueError("--hip_graph needs the pose network on its own stream (--pose_streams 1)")
        sync = getattr(self.opt, "grad_sync", "auto")
        if sync == "auto":
            sync = "flat" if self.use_graph else "ddp"
        if self.use_graph and sync == "ddp" and world_size > 1:
            raise ValueError("--hip_graph needs --grad_sync flat (DDP hooks are not graph-capturable)")
        streams = ([torch.cuda.current_stream(self.device), self._pose_stream]
                   if self._pose_stream is not None else None)
        self.ddp = wrap_ddp(self.nets, self.device, streams) if (world_size > 1 and sync == "ddp") else None
        # one GPU needs no buckets: under capture the gradients are allocated (and
        # freed) in the graph's private pool like every other tensor, at the same
        # addresses on every replay, and autograd hands each producer's output over
        # instead of adding it into a pre-zeroed bucket (~150 add launches per step).
        # An explicit --grad_sync flat builds them anyway (buckets, communication
        # stream, stream waits and copies, no collective at world size 1): the
        # multi-GPU graph path exercised on one GPU.
        explicit_flat = getattr(self.opt, "grad_sync", "auto") == "flat"
        self.flat_sync = FlatGradSync(self.nets.named_parameters(), world_size) \
            if ((world_size > 1 and (sync == "flat" or self.use_graph)) or explicit_flat) else None
        self.graph = None
        self.seed_tensor = None
        self._choices_agreed = False

        # Adam (trainer.py:102): one HIP launch per step over every parameter (optim.py);
        # under hipGraph its capturable form: the lr is a device tensor that StepLR
        # updates in place (lr_scheduler._update_param_group_val -> fill_), so replays
        # see the decay, and the step counter lives on the device
        if self.device.type == "cuda":
            self.model_optimizer = FusedAdam(self.parameters_to_train, self.opt.learning_rate,
                                             capturable=self.use_graph)
            if (self.use_graph and world_size == 1 and self.flat_sync is None and self._pose_stream is not None
                    and self.use_pose_net and self.opt.pose_model_type == "separate_resnet"
                    and os.environ.get("MD2_ADAM_SPLIT", "1") != "0"):
                # one GPU (no gradient averaging between the backward and the update): the
                # pose networks' parameters — the tail of parameters_to_train — update on
                # the stream that produced their gradients.  Not with FlatGradSync: its
                # buckets are filled on the communication stream, which only the main
                # stream joins (sync())
                pose_params = [p for n in ("pose_encoder", "pose") if n in self.models
                               for p in self.models[n].parameters()]
                self.model_optimizer.split = (self._pose_stream, pose_params)
        else:
            self.model_optimizer = optim.Adam(self.parameters_to_train, self.opt.learning_rate)
        self._adam_split = getattr(self.model_optimizer, "split", None) is not None
        self.model_lr_scheduler = optim.lr_scheduler.StepLR(self.model_optimizer, self.opt.scheduler_step_size, 0.1)
        if self.opt.load_weights_folder is not None:
            self.load_model()

        self.src_frames = list(self.opt.frame_ids[1:])
        self.hot = HotPathConfig(
            batch=self.opt.batch_size, height=self.opt.height, width=self.opt.width,
            num_src=len(self.src_frames), num_scales=self.num_scales, min_depth=self.opt.min_depth,
            max_depth=self.opt.max_depth, disparity_smoothness=self.opt.disparity_smoothness,
            no_ssim=self.opt.no_ssim, avg_reprojection=self.opt.avg_reprojection,
            disable_automasking=self.opt.disable_automasking, v1_multiscale=self.opt.v1_multiscale,
            t_per_scale=self.opt.pose_model_type == "posecnn", predictive_mask=bool(self.opt.predictive_mask))
        self.noise_override = None   # {scale: unit-normal noise}; tests pin the tie-break noise with it
        self.depth_metric_names = ["de/abs_rel", "de/sq_rel", "de/rms", "de/log_rms", "da/a1", "da/a2", "da/a3"]
        self.epoch = 0
        self.step = 0

    # ------------------------------------------------------------------ modes
    def set_train(self):
        for m in self.models.values():
            m.train()

    def set_eval(self):
        for m in self.models.values():
            m.eval()

    # ------------------------------------------------------------- networks
    def _run_networks(self, models, inputs):
        """Encoder, depth decoder and pose networks (trainer.py:234-255).  With
        --amp bf16 they run under bf16 autocast and their outputs are cast back to
        fp32 for the (fp32) photometric loss."""
        amp = getattr(self.opt, "amp", "none") == "bf16"
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp and self.device.type == "cuda"):
            outputs = self._networks_body(models, inputs)
        if amp:
            outputs = _to_fp32(outputs)
        return outputs

    def _networks_body(self, models, inputs):
        # The pose network does not read the depth network (except pose_model_type
        # "shared"): it runs on a second HIP stream so the two overlap; autograd runs
        # its backward on that stream too.
        side = self._pose_stream if (self.use_pose_net and self.opt.pose_model_type != "shared") else None
        main = torch.cuda.current_stream(self.device) if side is not None else None
        pose_out = None
        # Autograd enqueues ready nodes newest-first, so the network whose forward is
        # enqueued LAST has its backward enqueued FIRST.  pose_last: the pose network
        # goes second, its backward (needing only dL/dT from the loss) goes onto its
        # stream before the host spends its time enqueuing the depth backward.
        pose_last = side is not None and (getattr(self, "pose_last", False) or _POSE_LAST)
        inputs_ready = None
        if pose_last:   # the pose stream waits for the inputs only, not the depth forward
            inputs_ready = torch.cuda.Event()
            inputs_ready.record(main)
        if side is not None and not pose_last:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                pose_out = self.predict_poses(inputs, None, models)
        if self.opt.pose_model_type == "shared":
            all_color_aug = torch.cat([inputs[("color_aug", i, 0)] for i in self.opt.frame_ids])
            all_features = models["encoder"](all_color_aug)
            all_features = [torch.split(f, self.opt.batch_size) for f in all_features]
            features = {k: [f[i] for f in all_features] for i, k in enumerate(self.opt.frame_ids)}
            outputs = models["depth"](features[0])
        else:
            features = models["encoder"](inputs["color_aug", 0, 0])
            outputs = models["depth"](features)
        if self.opt.predictive_mask:
            outputs["predictive_mask"] = models["predictive_mask"](
                features[0] if isinstance(features, dict) else features)
        if pose_last:
            side.wait_event(inputs_ready)
            with torch.cuda.stream(side):
                pose_out = self.predict_poses(inputs, None, models)
        if self.use_pose_net:
            if side is not None:
                main.wait_stream(side)
                for v in pose_out.values():
                    v.record_stream(main)
            else:
                pose_out = self.predict_poses(inputs, features, models)
            outputs.update(pose_out)
        return outputs

    def predict_poses(self, inputs, features, models=None):
        """trainer.py:262-318; all cam_T_cam of the step come from one fused launch
        (pose_ops.poses_to_transforms, the transformation_from_parameters of
        trainer.py:294-295 / 315-316)."""
        models = models if models is not None else self.models
        outputs = {}
        aas, trs, invs, fids = [], [], [], []
        packed = None   # (F,B,6) pose-decoder output when every frame came from one batched call
        if self.num_pose_frames == 2:
            if self.opt.pose_model_type == "shared":
                pose_feats = {f_i: features[f_i] for f_i in self.opt.frame_ids}
            else:
                pose_feats = {f_i: inputs["color_aug", f_i, 0] for f_i in self.opt.frame_ids}
            temporal = [f_i for f_i in self.opt.frame_ids[1:] if f_i != "s"]
            pairs = [[pose_feats[f_i], pose_feats[0]] if f_i < 0 else [pose_feats[0], pose_feats[f_i]]
                     for f_i in temporal]
            if (self.opt.pose_model_type == "separate_resnet" and len(temporal) > 1 and self.device.type == "cuda"
                    and self.batch_pose_pairs):
                # every pair through the pose network as ONE batch; BatchNorm keeps per-pair
                # statistics (bn_groups), so this equals the reference's one call per pair
                B = self.opt.batch_size
                # the (pairs*B, 6, H, W) normalised encoder input in one pass, straight
                # into the encoder's layout (ResnetEncoder.prepare); the frames are data
                enc = models["pose_encoder"]
                x = enc.prepare(pairs)
                with bn_groups(len(temporal)):
                    feats = enc.forward_prepared(x)
                dec = getattr(models["pose"], "module", models["pose"])   # DDP-wrapped or not
                dec.packed_output = True
                try:
                    x6 = models["pose"]([feats])                        # (pairs*B, frames, 1, 6)
                finally:
                    dec.packed_output = False
                axisangle_all, translation_all = x6[..., :3], x6[..., 3:]
                per_pair = [(axisangle_all[i * B:(i + 1) * B], translation_all[i * B:(i + 1) * B])
                            for i in range(len(temporal))]
                if x6.dtype == torch.float32:   # the first predicted frame, as axisangle[:, 0] below
                    packed = x6[:, 0, 0].view(len(temporal), B, 6)
            else:
                per_pair = []
                for pair in pairs:
                    if self.opt.pose_model_type == "separate_resnet":
                        pair = [models["pose_encoder"](torch.cat(pair, 1))]
                    elif self.opt.pose_model_type == "posecnn":
                        pair = torch.cat(pair, 1)
                    per_pair.append(models["pose"](pair))
            for f_i, (axisangle, translation) in zip(temporal, per_pair):
                outputs[("axisangle", 0, f_i)] = axisangle
                outputs[("translation", 0, f_i)] = translation
                aas.append(axisangle[:, 0, 0])
                trs.append(translation[:, 0, 0])
                invs.append(f_i < 0)
                fids.append(f_i)
        else:
            if self.opt.pose_model_type in ["separate_resnet", "posecnn"]:
                pose_inputs = torch.cat([inputs[("color_aug", i, 0)] for i in self.opt.frame_ids if i != "s"], 1)
                if self.opt.pose_model_type == "separate_resnet":
                    pose_inputs = [models["pose_encoder"](pose_inputs)]
            else:
                pose_inputs = [features[i] for i in self.opt.frame_ids if i != "s"]
            axisangle, translation = models["pose"](pose_inputs)
            for i, f_i in enumerate(self.opt.frame_ids[1:]):
                if f_i != "s":
                    outputs[("axisangle", 0, f_i)] = axisangle
                    outputs[("translation", 0, f_i)] = translation
                    aas.append(axisangle[:, i, 0])
                    trs.append(translation[:, i, 0])
                    invs.append(False)
                    fids.append(f_i)
        self._T_all = None
        if fids:
            if packed is not None:
                T = packed_poses_to_transforms(packed, invs)
            else:
                T = poses_to_transforms(torch.stack(aas).float(), torch.stack(trs).float(), invs)
            for i, f_i in enumerate(fids):
                outputs[("cam_T_cam", 0, f_i)] = T[i]
            self._T_all = (T, tuple(fids))
        return outputs

    # ------------------------------------------------------------- hot path
    def _colors(self, inputs):
        cols = []
        for s in range(self.num_scales):
            row = [inputs[("color", 0, s)]]
            for f in self.src_frames:
                row.append(inputs.get(("color", f, s)) if (self.opt.v1_multiscale or s == 0) else None)
            cols.append(row)
        return cols

    def _intrinsics(self, inputs):
        K = [inputs[("K", s)] for s in range(self.num_scales)]
        inv_K = [inputs[("inv_K", s)] for s in range(self.num_scales)]
        return K, inv_K

    def _stacked_T(self, inputs, outputs):
        """(S,B,4,4) cam_T_cam in frame order (trainer.py:360-363); posecnn: per scale
        (num_scales,S,B,4,4) with the translation rescaled by mean inverse depth
        (trainer.py:366-375)."""
        if self.opt.pose_model_type != "posecnn":
            Ts = [inputs["stereo_T"] if f == "s" else outputs[("cam_T_cam", 0, f)] for f in self.src_frames]
            T_all = getattr(self, "_T_all", None)
            if (T_all is not None and T_all[1] == tuple(self.src_frames)
                    and all(t._base is T_all[0] and t.storage_offset() == i * T_all[0].stride(0)
                            for i, t in enumerate(Ts))):
                return T_all[0]    # the fused producer's (S,B,4,4) already is the stack
            return torch.stack(Ts, 0)
        temporal = [f for f in self.src_frames if f != "s"]
        return posecnn_transforms([outputs[("disp", s)] for s in range(self.num_scales)],
                                  torch.stack([outputs[("axisangle", 0, f)][:, 0, 0] for f in temporal]),
                                  torch.stack([outputs[("translation", 0, f)][:, 0, 0] for f in temporal]),
                                  self.src_frames, inputs.get("stereo_T"), self.opt.height, self.opt.width,
                                  self.opt.min_depth, self.opt.max_depth, self.opt.v1_multiscale)

    def generate_images_pred(self, inputs, outputs):
        """Materialise what trainer.py:341-391 writes into `outputs` (no autograd)."""
        K, inv_K = self._intrinsics(inputs)
        with torch.no_grad():
            T = self._stacked_T(inputs, outputs)
            if self.hot.t_per_scale:
                T = T[0]  # the materialised images use the scale-0 pose (logging only)
                cfg = HotPathConfig(**{**self.hot.__dict__, "t_per_scale": False})
            else:
                cfg = self.hot
            res = generate_images(cfg, [outputs[("disp", s)].detach() for s in range(self.num_scales)],
                                  self._colors(inputs), K, inv_K, T.detach())
        for s in range(self.num_scales):
            outputs[("depth", 0, s)] = res["depth"][s]
            src_s = s if self.opt.v1_multiscale else 0
            for fi, f in enumerate(self.src_frames):
                outputs[("sample", f, s)] = res["sample"][(fi, s)]
                outputs[("color", f, s)] = res["color"][(fi, s)]
                if not self.opt.disable_automasking:
                    outputs[("color_identity", f, s)] = inputs[("color", f, src_s)]

    def compute_losses(self, inputs, outputs):
        """trainer.py:407-496 (+ the warp of 341-391) as one fused HIP op."""
        K, inv_K = self._intrinsics(inputs)
        T = self._stacked_T(inputs, outputs)
        if self.seed_tensor is not None:   # graph replay: the step counter lives on the device
            seed = int(self.opt.noise_seed) * 1000003 * 131 + self.rank
        else:
            seed = (int(self.opt.noise_seed) * 1000003 + self.step) * 131 + self.rank
        mask, bce = None, None
        if self.hot.predictive_mask:
            mask, bce = predictive_mask_inputs(self.hot, {s: outputs["predictive_mask"][("disp", s)]
                                                          for s in range(self.num_scales)})
        loss_vec, sel = photometric_loss(self.hot, [outputs[("disp", s)] for s in range(self.num_scales)],
                                         self._colors(inputs), K, inv_K, T, noise=self.noise_override,
                                         seed=seed, seed_tensor=self.seed_tensor, mask=mask,
                                         src8=inputs.get("color_src8"))
        if bce is not None:   # trainer.py:457-459: loss/s += 0.2 * BCE(mask, 1)
            loss_vec = loss_vec + torch.cat([bce, bce.mean().view(1)])
        losses = {"loss/{}".format(s): loss_vec[s] for s in range(self.num_scales)}
        losses["loss"] = loss_vec[self.num_scales]
        if not self.opt.disable_automasking:
            # trainer.py:481-482, all scales in one compare + one cast over the packed map.
            # Logging-only: inside a training step it runs on the pose stream, which idles
            # here until the hot path's backward hands it dL/dT, instead of delaying that
            # backward on the main stream (_step_body joins the pose stream after backward)
            C = self.hot.noise_channels()
            side = (self._pose_stream if (self._in_step and self.use_pose_net and _LOGMAPS_SIDE) else None)
            if side is not None:
                main = torch.cuda.current_stream(self.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    maps = selection_maps(self.hot, sel.gt(C - 1).float())
                sel.record_stream(side)
                for m in maps.values():
                    m.record_stream(main)
            else:
                maps = selection_maps(self.hot, sel.gt(C - 1).float())
            for s, m in maps.items():
                outputs["identity_selection/{}".format(s)] = m
        return losses

    def process_batch(self, inputs):
        """trainer.py:228-260."""
        for key, ipt in inputs.items():
            if ipt.device != self.device:
                inputs[key] = ipt.to(self.device, non_blocking=True)
        nets = self.ddp if self.ddp is not None else self.nets
        outputs = nets(self, inputs)
        if self.opt.materialize_images:
            self.generate_images_pred(inputs, outputs)
        losses = self.compute_losses(inputs, outputs)
        return outputs, losses

    def _step_body(self, inputs):
        """process_batch + backward + gradient averaging + Adam (trainer.py:205-209).
        The conv weights' split-bf16 planes are refreshed once for the whole step
        (conv_ops.PlaneBank, one launch) and valid until the optimizer step — under
        --amp bf16 the bf16-rounded weights of the bf16 convolutions likewise."""
        bank = self.device.type == "cuda" and conv_ops.PLANE_BANK
        if bank:
            conv_ops.begin_step(self.device, bf16=getattr(self.opt, "amp", "none") == "bf16")
        self._in_step = True
        if self._adam_split:
            # the optimizer's step counter and bias corrections first, so that the pose
            # network's parameters update on the pose stream as soon as its backward is
            # done, while the depth network's backward still runs (FusedAdam.split)
            self.model_optimizer.prepare_step()
        try:
            outputs, losses = self.process_batch(inputs)
            if self.flat_sync is not None:
                self.flat_sync.zero()
            else:
                self.model_optimizer.zero_grad(set_to_none=True)
            if _JOIN_BEFORE_BWD and self._pose_stream is not None and self.use_pose_net:
                self._pose_stream.wait_stream(torch.cuda.current_stream(self.device))
            losses["loss"].backward()
            if self._pose_stream is not None and self.use_pose_net:
                # the pose stream's work of this step (its backward, the logging maps of
                # compute_losses) joined before anything reads it
                torch.cuda.current_stream(self.device).wait_stream(self._pose_stream)
        finally:
            self._in_step = False
            if bank:
                conv_ops.end_step()
        if self.flat_sync is not None:
            self.flat_sync.sync()
        self.model_optimizer.step()
        if self.seed_tensor is not None:
            self.seed_tensor.add_(1)
        return outputs, losses

    def eager_step(self, inputs):
        """One training step run eagerly (not replayed).  After a capture it runs on the
        capture's stream: every parameter's AccumulateGrad node was created there (at the
        warm-up) and keeps that stream, so a step issued on another stream would make
        autograd accumulate across streams (its stream-mismatch warning)."""
        side = getattr(self, "graph_stream", None)
        if side is None:
            return self._step_body(inputs)
        cur = torch.cuda.current_stream(self.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            out = self._step_body(inputs)
        cur.wait_stream(side)
        return out

    def _capture(self, inputs, warmup: int = 3):
        """Capture one whole training step (networks, fused hot path, backward,
        all-reduce, Adam) into a hipGraph; later steps replay it.

        The warm-up runs (allocator pools, MIOpen solver choice, lazily created Adam
        state) are real steps, so everything they advance — parameters, Adam moments
        and step counters, BatchNorm running statistics, the noise seed — is put back
        before the capture: the first replay is then exactly the first eager step."""
        self.static_inputs = {k: v.to(self.device).clone() for k, v in inputs.items()}
        self.seed_tensor = torch.zeros(1, dtype=torch.int64, device=self.device)
        snap = self._training_state()
        if self.flat_sync is not None:
            self.flat_sync.recalibrate()   # the warm-up's first step measures the send order
        side = torch.cuda.Stream(self.device)
        self.graph_stream = side   # an eager step after the capture runs here too (eager_step)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._step_body(self.static_inputs)
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._agree_conv_choices()   # before the capture: the graph holds rank 0's kernels
        self._restore_training_state(snap)
        self.graph = torch.cuda.CUDAGraph()
        dot = os.environ.get("MD2_GRAPH_DOT")
        if dot:
            self.graph.enable_debug_mode()
        # capture on the warm-up's stream: a parameter's AccumulateGrad node is created
        # once and keeps the stream of its first backward, so capturing on torch's own
        # capture stream after warming up on `side` made autograd accumulate those
        # gradients across streams (its "AccumulateGrad node's stream does not match"
        # warning at the capture; variants of this step traced 60 of 88 main-network
        # parameters on the warm-up stream during the capture)
        with torch.cuda.graph(self.graph, stream=side):
            self.static_outputs, self.static_losses = self._step_body(self.static_inputs)
        if dot:
            self.graph.debug_dump(dot)

    def _agree_conv_choices(self, again: bool = False):
        """After the first step's convolution autotune (conv_ops._fastest times its
        candidates on each rank without any collective): every rank adopts one per-shape
        table (conv_ops.agree_choices: the union of the ranks' choices, rank 0's first),
        at a point where every rank is present and none is inside a forward or backward.
        `again` (the end of every epoch, run_epoch): once more, for shapes any rank met
        after the first agreement — one all_gather of small tables, never inside a
        capture."""
        if self.world_size > 1 and (again or not self._choices_agreed):
            conv_ops.agree_choices()
            self._choices_agreed = True

    def _training_state(self):
        """Copies of every tensor a training step advances (see _capture)."""
        with torch.no_grad():
            params = [p.detach().clone() for p in self.parameters_to_train]
            bufs = [b.detach().clone() for m in self.models.values() for b in m.buffers()]
            opt = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                   for p, st in self.model_optimizer.state.items()}
        return params, bufs, opt

    def _restore_training_state(self, snap):
        """In place (the graph captures these storages): parameters and buffers back
        to the snapshot; Adam state back to the snapshot, or to its initial value
        (zero moments, step 0) where the warm-up created it."""
        params, bufs, opt = snap
        with torch.no_grad():
            for p, v in zip(self.parameters_to_train, params):
                p.copy_(v)
            for b, v in zip((b for m in self.models.values() for b in m.buffers()), bufs):
                b.copy_(v)
            for p, st in self.model_optimizer.state.items():
                old = opt.get(id(p))
                for k, v in st.items():
                    if not torch.is_tensor(v):
                        continue
                    if old is not None and k in old:
                        v.copy_(old[k])
                    else:
                        v.zero_()
            self.seed_tensor.zero_()

    def _bn_state(self):
        """Restore the folded BatchNorm counters (checkpoint key parity)."""
        for m, k in zip(self._bn_layers, self._bn_mult):
            m.num_batches_tracked = torch.tensor(self._bn_steps * k, dtype=torch.long, device=self.device)

    def _bn_fold(self):
        for m in self._bn_layers:
            m.num_batches_tracked = None

    def train_step(self, inputs):
        """One optimisation step (trainer.py:205-209)."""
        self._bn_steps += 1
        if not self.use_graph:
            outputs, losses = self._step_body(inputs)
            self.step += 1
            self._agree_conv_choices()
            return outputs, losses
        if self.graph is None:
            self._capture(inputs)
        else:
            for k, v in inputs.items():
                dst = self.static_inputs[k]
                if v.data_ptr() != dst.data_ptr():
                    dst.copy_(v, non_blocking=True)
        self.graph.replay()
        self.step += 1
        return self.static_outputs, self.static_losses

    def run_epoch(self, batches: Iterable, log_every: int = 0):
        self.set_train()
        for batch_idx, inputs in enumerate(batches):
            t0 = time.time()
            outputs, losses = self.train_step(inputs)
            if log_every and batch_idx % log_every == 0:
                loss = float(losses["loss"])
                self.log_time(batch_idx, time.time() - t0, loss)
        self.model_lr_scheduler.step()
        self.epoch += 1
        self._agree_conv_choices(again=True)

    def compute_depth_losses(self, inputs, outputs, losses):
        """trainer.py:498-526 (monitoring only)."""
        depth_pred = outputs[("depth", 0, 0)]
        depth_pred = torch.clamp(F.interpolate(depth_pred, [375, 1242], mode="bilinear", align_corners=False),
                                 1e-3, 80).detach()
        depth_gt = inputs["depth_gt"]
        mask = depth_gt > 0
        crop = torch.zeros_like(mask)
        crop[:, :, 153:371, 44:1197] = 1
        mask = mask * crop
        depth_gt = depth_gt[mask]
        depth_pred = depth_pred[mask]
        depth_pred *= torch.median(depth_gt) / torch.median(depth_pred)
        depth_pred = torch.clamp(depth_pred, min=1e-3, max=80)
        for name, v in zip(self.depth_metric_names, compute_depth_errors(depth_gt, depth_pred)):
            losses[name] = np.array(v.cpu())

    def log_time(self, batch_idx, duration, loss):
        print("epoch {:>3} | batch {:>6} | examples/s: {:5.1f} | loss: {:.5f}".format(
            self.epoch, batch_idx, self.opt.batch_size * self.world_size / max(duration, 1e-9), loss))

    # -------------------------------------------------------- checkpoints
    def save_opts(self):
        models_dir = os.path.join(self.log_path, "models")
        os.makedirs(models_dir, exist_ok=True)
        with open(os.path.join(models_dir, "opt.json"), "w") as f:
            json.dump(self.opt.__dict__.copy(), f, indent=2)

    def save_model(self):
        """trainer.py:585-603: weights_{epoch}/{model}.pth + adam.pth."""
        folder = os.path.join(self.log_path, "models", "weights_{}".format(self.epoch))
        os.makedirs(folder, exist_ok=True)
        self._bn_state()
        for name, model in self.models.items():
            state = model.state_dict()
            if name == "encoder":
                state["height"] = self.opt.height
                state["width"] = self.opt.width
                state["use_stereo"] = self.opt.use_stereo
            torch.save(state, os.path.join(folder, "{}.pth".format(name)))
        torch.save(self.model_optimizer.state_dict(), os.path.join(folder, "adam.pth"))
        self._bn_fold()
        return folder

    def load_model(self):
        """trainer.py:605-630 (safe loader: weights_only=True)."""
        folder = os.path.expanduser(self.opt.load_weights_folder)
        assert os.path.isdir(folder), "Cannot find folder {}".format(folder)
        self._bn_state()
        for n in self.opt.models_to_load:
            if n not in self.models:
                continue
            model_dict = self.models[n].state_dict()
            loaded = torch.load(os.path.join(folder, "{}.pth".format(n)), map_location=self.device,
                                weights_only=True)
            model_dict.update({k: v for k, v in loaded.items() if k in model_dict})
            self.models[n].load_state_dict(model_dict)
        if self._bn_layers:
            self._bn_steps = int(self._bn_layers[0].num_batches_tracked) // self._bn_mult[0]
        self._bn_fold()
        adam = os.path.join(folder, "adam.pth")
        if os.path.isfile(adam):
            self.model_optimizer.load_state_dict(torch.load(adam, map_location=self.device, weights_only=True))
