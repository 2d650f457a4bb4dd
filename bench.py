"""Training throughput benchmark (BASELINE.json metric: training images/sec at
640x192 mono, 1/2/4/8 GPUs; loss delta vs reference).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (configs[1] of BASELINE.json): mono 640x192, ResNet-18 depth encoder +
DepthDecoder + separate ResNet-18 pose encoder + PoseDecoder, frame_ids [0,-1,1],
batch 12 per GPU, fp32, Adam step — one full `Trainer.train_step` per step, with
the photometric hot path (warp + SSIM/L1 + min-reprojection + smoothness, fwd+bwd)
in the fused HIP kernels.  Synthetic KITTI-shaped inputs resident in HBM, random
init weights (no network for ImageNet weights).  Data parallel: one process per
GPU, each with its own 12-image shard (weak scaling), DDP gradient all-reduce over
RCCL.  Rank 0 prints ONE JSON line.

Extra fields:
  roofline      — the fused hot path (md2_photometric_fwd + md2_photometric_bwd: every
                  kernel of it), HIP-event timed on its launch stream during the timed
                  steps (first kernel's start to last kernel's end of each call).
                  Algorithmic work per step from monodepth2_amd/roofline.py (SURVEY.md
                  §8(d)): bytes = B * 4 N (3 S + 6.640625), flops = B * N * the pinned
                  per-pixel census; both fractions are reported (HBM vs 8 TB/s, VALU vs
                  the 157.3 TF FP32 vector peak) and the larger, binding one is the
                  headline.  traffic = HBM bytes per step measured IN THIS RUN by two
                  rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; FETCH x2 per
                  MI355X_MICROARCH.md) over tools/hot_bench.py at the same shape
                  (rank 0, N=1; --pmc 0 skips them).  `photo_bwd` details the
                  dominant single kernel.
  cpu_baseline  — rank 0, N=1: the same training step on the host cores with the
                  oracle hot path (oracle/md2_oracle.py, op-for-op restatement of
                  the reference), a bounded sample of steps at batch 4 (configs[0]).
  loss_delta_vs_oracle — |loss_GPU - loss_oracle| on identical inputs, weights and
                  tie-break noise (first step).
  eager_aten_hot_path_ms — configs[1]'s own comparison: the reference's hot path
                  (generate_images_pred + compute_losses, trainer.py:341-496) as eager
                  ATen ops on the same GPU, fwd+bwd on the step's own outputs; the
                  ratio to the HIP hot path is context, never the target.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# MIOpen: FAST find mode = tuned find-db hits (monodepth2_amd/miopen_db) or the
# immediate-mode heuristic, never an exhaustive search (see monodepth2_amd/__init__.py)
if "--miopen-find" in sys.argv:
    os.environ["MIOPEN_FIND_MODE"] = sys.argv[sys.argv.index("--miopen-find") + 1].upper()
import monodepth2_amd  # noqa: E402,F401  (sets the MIOpen environment before torch loads MIOpen)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec at 640x192 mono, 1/2/4/8 GPUs; loss delta vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, HBM3E spec
F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, dense f32 matrix (= f32 vector) peak
F32_VALU_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, "Peak FP32 (vector)"
BF16_MFMA_PEAK_TFLOPS = 2500.0 # dense bf16; the split-bf16 convs issue 6 bf16 products per f32 product
ROUND = "r03"


HOT_KERNELS = "pack_src8|photo_|smooth_fwd|finalize_fwd|disp_grad|grad_T_kernel"


def pmc_traffic(args, S, timeout=150):
    """HBM bytes per hot-path step (forward + backward), measured now: two rocprofv3
    --pmc passes (FETCH_SIZE, WRITE_SIZE: one pass cannot hold both) over a short run
    of this same training step (bench.py --steps 3 at the same shape, so the caches
    hold what they hold in the timed steps), averaged per dispatch per kernel and
    summed over the hot path's kernels.  FETCH_SIZE x2 (gfx950 under-reports wide
    reads by half, MI355X_MICROARCH.md §HBM), KB -> bytes.  Runs in child processes
    while this one waits (no GPU work of its own in flight)."""
    import csv
    import glob
    import re
    import shutil
    import signal
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    per = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="md2pmc_", dir="/tmp")
        cmd = [exe, "--pmc", counter, "--kernel-include-regex", HOT_KERNELS, "-d", d, "-o", "pmc",
               "--output-format", "csv", "--", sys.executable, os.path.join(REPO, "bench.py"),
               "--batch", str(args.batch), "--height", str(args.height), "--width", str(args.width),
               "--num_layers", str(args.num_layers), "--amp", args.amp, "--steps", "3", "--warmup", "2",
               "--no-cpu-baseline", "--no-parity", "--pmc", "0", "--no-conv-roofline", "--no-eager-aten", "--graph", "0",
               "--src8", "0"] + \
              (["--stereo"] if args.stereo else [])
        env = dict(os.environ, TMPDIR="/tmp")
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, start_new_session=True)
        try:
            _, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.communicate()
            return None, f"rocprofv3 --pmc {counter} timed out"
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if p.returncode != 0 or not files:
            return None, f"rocprofv3 --pmc {counter} rc={p.returncode}: {err.decode(errors='replace')[-300:]}"
        vals = {}
        for f in files:
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == counter:
                    name = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Kernel_Name"]).split("(")[0].split("<")[0]
                    vals.setdefault(name, []).append(float(r["Counter_Value"]))
        per[counter] = {k: sum(v) / len(v) for k, v in vals.items()}
        shutil.rmtree(d, ignore_errors=True)
    kernels = sorted(set(per["FETCH_SIZE"]) | set(per["WRITE_SIZE"]))
    # raw = FETCH + WRITE; corrected = 2 FETCH + WRITE.  tools/fetch_calib.py measured on
    # MI355X (profiles/r04/fetch_calib.json): FETCH_SIZE counts half the bytes of 4-, 8-
    # and 16-B-per-lane reads alike (coalesced or one line per lane), WRITE_SIZE every
    # width exactly; 1- and 2-B-per-lane reads are not counted at all (the argmin-code
    # bytes the backward reads are missing from both figures)
    by_kernel = {k: {"raw": int(1024 * (per["FETCH_SIZE"].get(k, 0.0) + per["WRITE_SIZE"].get(k, 0.0))),
                     "corrected": int(1024 * (2 * per["FETCH_SIZE"].get(k, 0.0) + per["WRITE_SIZE"].get(k, 0.0))),
                     "write": int(1024 * per["WRITE_SIZE"].get(k, 0.0))}
                 for k in kernels}
    return by_kernel, None


_T0 = time.perf_counter()


def log(msg):
    if int(os.environ.get("RANK", 0)) == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=12, help="images per GPU")
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--num_layers", type=int, default=18)
    ap.add_argument("--stereo", action="store_true")
    ap.add_argument("--frame-ids", type=str, default="0,-1,1",
                    help="comma list (trainer --frame_ids): e.g. '0' with --stereo is the stereo-only step "
                         "(no pose network; an experiment, not the headline)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-conv-roofline", action="store_true")
    ap.add_argument("--no-eager-aten", action="store_true",
                    help="skip timing the reference's eager ATen hot path beside the HIP one")
    ap.add_argument("--pmc", type=int, default=1, help="measure the hot path's HBM traffic with rocprofv3 "
                    "PMC passes in this run (rank 0, N=1)")
    ap.add_argument("--cudnn-benchmark", action="store_true", help="MIOpen exhaustive find per conv shape")
    ap.add_argument("--deterministic", type=int, default=-1,
                    help="MIOpen deterministic algorithms (1/0; default: MIOpen's own choice — its deterministic "
                         "bf16 solvers take 9.4 s a step at B=32, DESIGN.md §6)")
    ap.add_argument("--channels-last", type=int, default=1, help="NHWC convolutions (1/0)")
    ap.add_argument("--pose-last", type=int, default=0,
                    help="1: pose network forward enqueued after the depth network (its backward first)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the whole step in a hipGraph (1/0; default: 1 on one GPU, where the captured "
                         "step is at or below eager and immune to a slow host, 0 with N > 1)")
    ap.add_argument("--pose-stream", type=int, default=1, help="pose network on its own HIP stream (1/0)")
    ap.add_argument("--miopen-find", type=str, default="fast", help="MIOPEN_FIND_MODE (fast|normal|...)")
    ap.add_argument("--amp", type=str, default="none", choices=["none", "bf16"],
                    help="bf16 autocast for the networks (config C5); the photometric loss stays fp32")
    ap.add_argument("--src8", type=int, default=1,
                    help="1: the batch carries the sources' 8-bit RGBx copies (color_src8), as the GPU input "
                         "pipeline writes them; 0: the hot path packs them from the fp32 colours every step")
    ap.add_argument("--gpu-augment", type=int, default=0,
                    help="1: every step also runs the input pipeline (flip + LANCZOS pyramid + jitter, "
                         "md2_aug_run) from resident 375x1242 uint8 frames")
    return ap.parse_args()


def make_trainer(args, device, rank, world):
    from monodepth2_amd.options import default_options
    from monodepth2_amd.trainer import Trainer
    opt = default_options(batch_size=args.batch, height=args.height, width=args.width,
                          num_layers=args.num_layers, weights_init="scratch", use_stereo=args.stereo,
                          frame_ids=[int(f) for f in args.frame_ids.split(",")], log_dir="/tmp/md2_bench",
                          channels_last=bool(args.channels_last), hip_graph=bool(args.graph), amp=args.amp,
                          pose_streams=args.pose_stream)
    tr = Trainer(opt, device=device, rank=rank, world_size=world)
    tr.pose_last = bool(args.pose_last)
    return tr


def loss_delta_vs_oracle(trainer, batch):
    """Same weights, inputs and noise: GPU fused hot path vs CPU oracle."""
    from monodepth2_amd.hotpath import photometric_loss
    from oracle.md2_oracle import HotPathOptions, hot_path
    with torch.no_grad():
        outputs = trainer.nets(trainer, batch)
    hot = trainer.hot
    gen = torch.Generator().manual_seed(1234)
    noise = {s: torch.randn(*hot.noise_shape(s), generator=gen) for s in range(hot.num_scales)}
    K, iK = trainer._intrinsics(batch)
    T = trainer._stacked_T(batch, outputs).detach()
    disps = [outputs[("disp", s)].detach() for s in range(hot.num_scales)]
    loss, _ = photometric_loss(hot, disps, trainer._colors(batch), K, iK, T,
                               noise={s: n.to(T.device) for s, n in noise.items()})
    cpu_inputs = {k: v.detach().cpu() for k, v in batch.items()}
    camT = {f: T[i].cpu() for i, f in enumerate(trainer.src_frames)}
    opt = HotPathOptions(height=hot.height, width=hot.width, frame_ids=trainer.opt.frame_ids)
    with torch.no_grad():
        ref, _ = hot_path(opt, {s: d.float().cpu() for s, d in enumerate(disps)}, cpu_inputs, camT, noise=noise,
                          keep_images=False)
    return abs(float(loss[hot.num_scales]) - float(ref["loss"]))


def time_hot_kernels(trainer, batch, n=10, src8=True):
    """Stand-alone fwd+bwd of the fused hot path on the step's own tensors, with the
    photometric kernels HIP-event timed (used when the step runs as a hipGraph,
    whose replays are not individually instrumented).  src8=False: without the
    loader's 8-bit source copies, i.e. with the forward's own pack pass."""
    from monodepth2_amd import _lib
    from monodepth2_amd.hotpath import photometric_loss
    with torch.no_grad():
        outputs = trainer.nets(trainer, batch)
    hot = trainer.hot
    K, iK = trainer._intrinsics(batch)
    T = trainer._stacked_T(batch, outputs).detach().requires_grad_(True)
    disps = [outputs[("disp", s)].detach().requires_grad_(True) for s in range(hot.num_scales)]
    colors = trainer._colors(batch)
    s8 = batch.get("color_src8") if src8 else None
    for _ in range(2):
        loss, _ = photometric_loss(hot, disps, colors, K, iK, T, seed=1, src8=s8)
        loss[hot.num_scales].backward()
    torch.cuda.synchronize()
    with _lib.KernelTimer(max_launches=4 * n + 8) as kt:
        for i in range(n):
            loss, _ = photometric_loss(hot, disps, colors, K, iK, T, seed=2 + i, src8=s8)
            loss[hot.num_scales].backward()
    return kt


def eager_aten_hot_path(trainer, batch, n=5):
    """configs[1]'s own comparison ("HIP warp+SSIM kernels vs PyTorch-ROCm
    grid_sample"): the reference's hot path as the reference writes it —
    generate_images_pred + compute_losses (trainer.py:341-496): per scale the bilinear
    upsample, disp_to_depth, BackprojectDepth / Project3D (bmm), F.grid_sample with
    border padding, the 3x3 SSIM of layers.py:218-248 + L1 for every reprojected AND
    every identity candidate (recomputed per scale, trainer.py:432-439), the 1e-5 randn
    tie-break, cat + torch.min, the mean-normalised smoothness — forward and backward to
    the disparities and the transforms, eagerly on PyTorch-ROCm (ATen's kernels), on the
    same GPU, the step's own network outputs, intrinsics and colours.  The layer objects
    are this package's restatement of the reference's layers.py (same signatures, same
    ATen ops), not the fused path.  HIP-event timed on torch's current stream (every op
    runs there); returns ms per fwd+bwd."""
    import torch.nn.functional as F
    from monodepth2_amd.layers import SSIM, BackprojectDepth, Project3D, disp_to_depth, get_smooth_loss
    o = trainer.opt
    with torch.no_grad():
        outputs = trainer.nets(trainer, batch)
    dev = batch[("color", 0, 0)].device
    B = batch[("color", 0, 0)].shape[0]
    nsc = trainer.num_scales
    ssim = SSIM().to(dev)
    backproject = BackprojectDepth(B, o.height, o.width).to(dev)
    project = Project3D(B, o.height, o.width).to(dev)
    T = trainer._stacked_T(batch, outputs).detach().requires_grad_(True)
    disps = [outputs[("disp", s)].detach().float().requires_grad_(True) for s in range(nsc)]
    srcs = trainer.src_frames

    def reproj_loss(pred, target):                                     # trainer.py:393-405
        l1 = (target - pred).abs().mean(1, True)
        return 0.85 * ssim(pred, target).mean(1, True) + 0.15 * l1

    def fwd_bwd():
        total = 0
        target = batch[("color", 0, 0)]
        for s in range(nsc):
            disp = F.interpolate(disps[s], [o.height, o.width], mode="bilinear", align_corners=False)
            _, depth = disp_to_depth(disp, o.min_depth, o.max_depth)  # trainer.py:350-354
            reproj = []
            for i, f in enumerate(srcs):                               # trainer.py:358-387
                pix = project(backproject(depth, batch[("inv_K", 0)]), batch[("K", 0)], T[i])
                warped = F.grid_sample(batch[("color", f, 0)], pix, padding_mode="border", align_corners=False)
                reproj.append(reproj_loss(warped, target))
            ident = torch.cat([reproj_loss(batch[("color", f, 0)], target) for f in srcs], 1)
            ident = ident + torch.randn(ident.shape, device=dev) * 0.00001   # trainer.py:468-469
            to_opt, _ = torch.min(torch.cat((ident, torch.cat(reproj, 1)), 1), dim=1)
            loss = to_opt.mean()
            norm = disps[s] / (disps[s].mean(2, True).mean(3, True) + 1e-7)  # trainer.py:486-490
            loss = loss + o.disparity_smoothness * get_smooth_loss(norm, batch[("color", 0, s)]) / (2 ** s)
            total = total + loss
        (total / nsc).backward()

    for _ in range(2):
        fwd_bwd()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fwd_bwd()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def conv_mfma_roofline(device):
    """The split-bf16 convolution (csrc/conv.hip conv_x6_kernel, the step's dominant
    hand-written MFMA kernel class) on the depth encoder's layer2 3x3 shape at B=12
    (M = 23,040 pixels, N = 128, K = 1,152), HIP-event timed on its stream: f32-class
    TFLOP/s against the f32 matrix peak, and the bf16 issue bound the six products
    per f32 product imply (2.5 PF / 6)."""
    from monodepth2_amd import conv_ops
    B, C, N, H, W = 12, 128, 128, 24, 80
    x = torch.randn(B, C, H, W, device=device).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(N, C, 3, 3, device=device) / 34.0).contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        conv_ops._fwd(x, w, 1, 1, conv_ops.X6)
    torch.cuda.synchronize()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        conv_ops._fwd(x, w, 1, 1, conv_ops.X6)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    flops = 2.0 * B * H * W * N * C * 9
    tf = flops / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "kernel": "conv_x6_kernel (split-bf16, f32-class)",
            "shape": f"fwd B={B} {C}->{N} 3x3 {H}x{W}", "achieved": round(tf, 1), "peak": F32_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(tf / F32_MFMA_PEAK_TFLOPS, 3),
            "bf16_issue_bound": round(BF16_MFMA_PEAK_TFLOPS / 6, 1), "avg_call_ms": round(ms, 4),
            "flops_per_call": int(flops)}


def cpu_baseline(args):
    """The reference-equivalent training step on the host CPU (oracle hot path)."""
    import torch.optim as optim
    from monodepth2_amd import networks
    from monodepth2_amd.data import synthetic_batch
    from monodepth2_amd.layers import transformation_from_parameters
    from oracle.md2_oracle import HotPathOptions, hot_path

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count()
    cores = max(1, min(cores, 16))   # the GPU box's CPU share is 16 cores
    torch.set_num_threads(cores)
    B, H, W = 4, args.height, args.width          # configs[0]: batch 4 on the CPU
    frame_ids = [0, -1, 1]
    enc = networks.ResnetEncoder(args.num_layers, False)
    dec = networks.DepthDecoder(enc.num_ch_enc, range(4))
    penc = networks.ResnetEncoder(args.num_layers, False, num_input_images=2)
    pdec = networks.PoseDecoder(penc.num_ch_enc, 1, 2)
    params = [p for m in (enc, dec, penc, pdec) for p in m.parameters()]
    adam = optim.Adam(params, 1e-4)
    inputs = synthetic_batch(B, H, W, frame_ids, 4, seed=5, eight_bit=True)
    opt = HotPathOptions(height=H, width=W, frame_ids=frame_ids)

    def step():
        outputs = dec(enc(inputs[("color_aug", 0, 0)]))
        camT = {}
        for f in frame_ids[1:]:
            pair = [inputs[("color_aug", f, 0)], inputs[("color_aug", 0, 0)]] if f < 0 else \
                [inputs[("color_aug", 0, 0)], inputs[("color_aug", f, 0)]]
            a, t = pdec([penc(torch.cat(pair, 1))])
            camT[f] = transformation_from_parameters(a[:, 0], t[:, 0], invert=(f < 0))
        losses, _ = hot_path(opt, {s: outputs[("disp", s)] for s in range(4)}, inputs, camT, keep_images=False)
        adam.zero_grad()
        losses["loss"].backward()
        adam.step()

    step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or n >= 50:
            break
    return {"value": round(B * n / el, 4), "unit": "images/s", "cores": cores, "kind": "port",
            "sample": f"{n} full training steps (R{args.num_layers} enc+dec+pose, oracle hot path, Adam) "
                      f"at batch {B}, {W}x{H}, fp32, torch CPU {cores} threads, {el:.1f} s"}


def make_augmenting_source(args, frame_ids, device, rank):
    """Per step: host draws (mono_dataset.py:136-179 order) + md2_aug_run over resident
    decoded frames, i.e. the reference DataLoader's per-item work on the GPU."""
    import random
    from monodepth2_amd.augment import GpuAugment, draw_item
    from monodepth2_amd.data import synthetic_batch
    Hn, Wn = 375, 1242
    nat = synthetic_batch(args.batch, Hn, Wn, frame_ids, 1, seed=300 + rank, device=device)
    frames = torch.stack([(nat[("color", f, 0)] * 255).round().to(torch.uint8).permute(0, 2, 3, 1)
                          for f in frame_ids]).contiguous()
    del nat
    aug = GpuAugment(args.height, args.width, Hn, Wn, frame_ids, args.batch, device=device)
    rng = random.Random(1000 + rank)
    return lambda: aug(frames, [draw_item(rng) for _ in range(args.batch)])


def main():
    args = parse()
    from monodepth2_amd.distributed import init_process_group
    from monodepth2_amd import _lib
    from monodepth2_amd.data import synthetic_batch

    rank, local_rank, world = init_process_group()
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    torch.backends.cudnn.benchmark = args.cudnn_benchmark
    if args.deterministic >= 0:
        torch.backends.cudnn.deterministic = bool(args.deterministic)
    _lib.lib()
    log(f"world={world} device={torch.cuda.get_device_name(device)}")

    if args.graph < 0:
        args.graph = 1 if world == 1 else 0
    try:
        trainer = make_trainer(args, device, rank, world)
    except ValueError as e:   # e.g. --graph 1 at N > 1 on a non-RCCL backend (Trainer refuses it)
        log(f"cannot run this configuration: {e}")
        if world > 1:
            dist.destroy_process_group()
        sys.exit(2)
    frame_ids = trainer.opt.frame_ids
    # colours as the reference's loader delivers them: uint8 frames through to_tensor,
    # i.e. exactly k/255 (datasets/mono_dataset.py:199-200)
    batch = synthetic_batch(args.batch, args.height, args.width, frame_ids, 4, seed=100 + rank, device=device,
                            eight_bit=True)
    if not args.src8:
        batch.pop("color_src8", None)
    next_batch = lambda: batch   # noqa: E731
    if args.gpu_augment:
        next_batch = make_augmenting_source(args, frame_ids, device, rank)
    log("trainer + batch ready")

    delta = None
    if not args.no_parity and rank == 0:
        delta = loss_delta_vs_oracle(trainer, batch)
        log(f"loss delta vs oracle = {delta:.3e}")

    import threading
    stop_hb = threading.Event()

    def heartbeat():
        while not stop_hb.wait(30.0):
            log("... still warming up (MIOpen solver search / kernel compilation)")
    threading.Thread(target=heartbeat, daemon=True).start()
    trainer.set_train()
    for i in range(args.warmup):
        t = time.perf_counter()
        trainer.train_step(next_batch())
        torch.cuda.synchronize()
        log(f"warmup step {i}: {1e3 * (time.perf_counter() - t):.1f} ms")
        if trainer.graph is not None and not args.gpu_augment:
            # the resident batch IS the captured step's input buffers (no per-replay copy)
            static = trainer.static_inputs
            next_batch = lambda: static   # noqa: E731
    stop_hb.set()
    torch.cuda.synchronize()
    # host enqueue rate: how long the CPU takes to issue 3 steps right after a sync
    # (<< 3 x ms_per_step means the GPU, not the launch path, bounds the step)
    t = time.perf_counter()
    for _ in range(3):
        trainer.train_step(next_batch())
    host_ms = 1e3 * (time.perf_counter() - t) / 3
    torch.cuda.synchronize()
    log(f"host enqueue time: {host_ms:.2f} ms/step")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    with _lib.KernelTimer(max_launches=8 * args.steps + 16) as kt:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            _, losses = trainer.train_step(next_batch())
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    final_loss = float(losses["loss"])

    timed_standalone = False
    if rank == 0 and kt.n_bwd == 0:
        kt = time_hot_kernels(trainer, batch)
        timed_standalone = True
        log("hot-path kernels timed stand-alone (graph mode)")
    if rank == 0:
        S = len(frame_ids) - 1
        B, H, W = args.batch, args.height, args.width
        bwd_ms = kt.bwd_ms / max(kt.n_bwd, 1)
        fwd_ms = kt.fwd_ms / max(kt.n_fwd, 1)
        fcall = kt.fwd_call_ms / max(kt.n_fwd_call, 1)
        bcall = kt.bwd_call_ms / max(kt.n_bwd_call, 1)
        hot_ms = fcall + bcall
        from monodepth2_amd.roofline import hot_path_census
        cen = hot_path_census(H, W, S)
        step_bytes, step_flops = B * cen.bytes, B * cen.flops
        gbs = step_bytes / (hot_ms * 1e-3) / 1e9
        tfs = step_flops / (hot_ms * 1e-3) / 1e12
        hbm_frac, valu_frac = gbs / HBM_PEAK_GBS, tfs / F32_VALU_PEAK_TFLOPS
        traffic, pmc_note, pmc_kernels, pack_traffic = None, "skipped (--pmc 0 or N>1)", None, None
        if args.pmc and world == 1:
            pmc_kernels, err = pmc_traffic(args, S)
            if pmc_kernels is not None:
                # the PMC child runs without the loader's 8-bit copies (--src8 0), so its
                # forward packs them (pack_src8_kernel); the other kernels read the same
                # RGBx dwords either way
                pack_traffic = sum(v["corrected"] for k, v in pmc_kernels.items() if k.startswith("pack_src8"))
                traffic = sum(v["corrected"] for k, v in pmc_kernels.items() if not k.startswith("pack_src8"))
                pmc_note = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes in this run over a 3-step run of this "
                            "training step (bench.py --steps 3); per dispatch, summed over the hot path's kernels: "
                            "2*FETCH+WRITE (KB->B), the x2 calibrated for the 4/8/16-B-per-lane reads these kernels "
                            "issue (tools/fetch_calib.py, profiles/r04/fetch_calib.json); raw = FETCH+WRITE per "
                            "kernel beside it")
            else:
                pmc_note = err
            log(f"pmc traffic: {traffic} B/step ({pmc_note[:80]})")
        # the sources' RGBx copies: handed in with the batch (md2_aug_run2 writes them as it
        # decodes; data.pack_rgbx for the resident bench batch), or packed by the forward
        # from the reference's fp32 colours (mono_dataset.py:199-200's to_tensor output):
        # that conversion timed beside the headline
        pack = None
        if "color_src8" in batch:
            k0, k1 = time_hot_kernels(trainer, batch, src8=False), time_hot_kernels(trainer, batch)
            pack_ms = max(k0.fwd_call_ms / max(k0.n_fwd_call, 1) - k1.fwd_call_ms / max(k1.n_fwd_call, 1), 0.0)
            hot_pack = hot_ms + pack_ms
            pack = {"src8": "loader", "pack_ms": round(pack_ms, 5),
                    "pack_timing": "fwd call without the loader's copies (pack_src8_kernel + the walk) minus "
                                   "the fwd call with them, stand-alone, same tensors",
                    "pack_traffic": pack_traffic,
                    "hot_path_ms_with_pack": round(hot_pack, 5),
                    "valu_frac_with_pack": round(step_flops / (hot_pack * 1e-3) / 1e12 / F32_VALU_PEAK_TFLOPS, 5),
                    "traffic_with_pack": (traffic + pack_traffic) if (traffic is not None and pack_traffic)
                    else None}
            log(f"src8 pack: {pack_ms:.4f} ms, {pack_traffic} B")
        head = ("valu", tfs, F32_VALU_PEAK_TFLOPS, "TFLOP/s", valu_frac) if valu_frac >= hbm_frac else \
            ("hbm", gbs, HBM_PEAK_GBS, "GB/s", hbm_frac)
        roof = {"bound": head[0], "kernel": "hot path: md2_photometric_fwd + md2_photometric_bwd (all their kernels)",
                "achieved": round(head[1], 3), "peak": head[2], "unit": head[3], "frac": round(head[4], 5),
                "traffic": traffic,
                "algorithmic_bytes_per_step": int(step_bytes), "algorithmic_flops_per_step": int(step_flops),
                "census": {"bytes_per_px": cen.bytes / (H * W), "fwd_flops_per_px": cen.fwd_flops / (H * W),
                           "bwd_flops_per_px": cen.bwd_flops / (H * W), "source": "monodepth2_amd/roofline.py"},
                "hbm": {"achieved_gbs": round(gbs, 2), "peak": HBM_PEAK_GBS, "frac": round(hbm_frac, 5)},
                "valu": {"achieved_tflops": round(tfs, 3), "peak": F32_VALU_PEAK_TFLOPS, "frac": round(valu_frac, 5)},
                "avg_ms_per_step": round(hot_ms, 5), "fwd_call_ms": round(fcall, 5), "bwd_call_ms": round(bcall, 5),
                "timing": ("stand-alone: HIP events on the step's own tensors right after the timed replays "
                           "(a captured step's kernels are not individually instrumented)" if timed_standalone
                           else "in the timed steps: HIP events the library stamps on each call's first and last "
                                "kernel, on the launch stream"),
                "calls": kt.n_bwd_call, "traffic_source": pmc_note, "traffic_by_kernel": pmc_kernels,
                "photo_bwd": {"avg_launch_ms": round(bwd_ms, 5), "launches": kt.n_bwd,
                              "share_of_hot_path": round(bwd_ms / hot_ms, 3) if hot_ms else None},
                "photo_fwd_kernels_ms": round(fwd_ms, 5)}
        if pack is not None:
            roof.update(pack)
        else:
            roof["src8"] = "packed in the forward (counted in the headline)"
        log(f"timed: {1e3 * dt / args.steps:.2f} ms/step, hot path {hot_ms:.3f} ms (fwd {fcall:.3f}, bwd {bcall:.3f};"
            f" photo_bwd {bwd_ms:.3f}), {tfs:.2f} TF = {valu_frac:.3f} of VALU peak, {gbs:.0f} GB/s, "
            f"adam table uploads {getattr(trainer.model_optimizer, 'rebuilds', '-')}")
        eager_ms = None
        if not args.no_eager_aten:
            eager_ms = eager_aten_hot_path(trainer, batch)
            log(f"eager ATen hot path (reference formulation): {eager_ms:.3f} ms fwd+bwd vs HIP {hot_ms:.3f} ms")
        conv_roof = None
        if not args.no_conv_roofline:
            conv_roof = conv_mfma_roofline(device)
            log(f"conv_x6: {conv_roof['achieved']} TFLOP/s ({conv_roof['frac']} of the f32 matrix peak)")
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args)
            log(f"cpu baseline: {cpu['value']} img/s")
        value = world * B * args.steps / dt
        line = {"metric": METRIC, "value": round(value, 3), "unit": "images/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "f32" if args.amp == "none" else "bf16 networks (autocast) + f32 photometric loss",
                "data": "synthetic (KITTI-shaped smooth textures as 8-bit k/255 colours like the loader's to_tensor output, random-init weights)",
                "config": {"workload": f"{'mono+stereo' if args.stereo else 'mono'}_{W}x{H} ResNet-{args.num_layers}"
                                       f" batch={B}/GPU full train step"
                                       + (" (configs[1])" if (not args.stereo and (W, H) == (640, 192)
                                                               and args.num_layers == 18 and args.amp == "none")
                                          else "")
                                       + (" + GPU input pipeline from 375x1242 uint8" if args.gpu_augment else ""),
                           "global_batch": B * world, "height": H, "width": W, "frame_ids": [str(f) for f in frame_ids],
                           "parallelism": f"dp{world}",
                           "step": "hipgraph replay" if trainer.graph is not None else "eager"},
                "roofline": roof, "conv_roofline": conv_roof, "cpu_baseline": cpu,
                "eager_aten_hot_path_ms": round(eager_ms, 4) if eager_ms is not None else None,
                "eager_aten_vs_hip_hot_path": ({
                    "eager_ms": round(eager_ms, 4), "hip_ms": round(hot_ms, 5),
                    "ratio": round(eager_ms / hot_ms, 2),
                    "what": "configs[1]'s comparison, context only (never the target): the reference's "
                            "generate_images_pred + compute_losses (trainer.py:341-496) as ATen ops "
                            "(grid_sample, avg_pool SSIM, min, smoothness) fwd+bwd on PyTorch-ROCm vs the HIP "
                            "hot path (roofline.avg_ms_per_step), same GPU, same run, same B=%d inputs, the "
                            "step's own disparities and transforms" % B} if eager_ms is not None else None),
                "loss_delta_vs_oracle": delta, "final_loss": round(final_loss, 6),
                "host_enqueue_ms_per_step": round(host_ms, 3)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
