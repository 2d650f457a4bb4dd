"""Trainer-level GPU tests: full training steps through the fused HIP hot path for
every option combination the reference supports, loss parity with the oracle on the
step's own network outputs, and the reference checkpoint layout."""
import os

import numpy as np
import pytest
import torch

from monodepth2_amd.data import synthetic_batch
from monodepth2_amd.options import default_options

pytestmark = pytest.mark.gpu

H, W, B = 64, 128, 2

CONFIGS = {
    "mono": {},
    "stereo": {"use_stereo": True},
    "stereo_only": {"use_stereo": True, "frame_ids": [0]},
    "no_ssim": {"no_ssim": True},
    "avg_reprojection": {"avg_reprojection": True},
    "no_automask": {"disable_automasking": True},
    "predictive_mask": {"disable_automasking": True, "predictive_mask": True},
    "v1_multiscale": {"v1_multiscale": True},
    "posecnn": {"pose_model_type": "posecnn"},
    "shared": {"pose_model_type": "shared"},
    "pose_all": {"pose_model_input": "all"},
    "resnet50": {"num_layers": 50},
    "mono_nchw": {"channels_last": 0},
    "amp_bf16": {"amp": "bf16"},
}


def make(name, **extra):
    from monodepth2_amd.trainer import Trainer
    kw = dict(batch_size=B, height=H, width=W, weights_init="scratch", log_dir="/tmp/md2_test",
              frame_ids=[0, -1, 1])
    kw.update(CONFIGS[name])
    kw.update(extra)
    torch.manual_seed(0)
    tr = Trainer(default_options(**kw), device=torch.device("cuda", 0))
    batch = synthetic_batch(B, H, W, tr.opt.frame_ids, 4, seed=3, device="cuda")
    return tr, batch


@pytest.mark.parametrize("name", list(CONFIGS))
def test_train_step_runs_and_updates(name):
    tr, batch = make(name)
    before = {n: p.detach().clone() for n, p in tr.nets.named_parameters()}
    losses = []
    for _ in range(3):
        _, l = tr.train_step(batch)
        losses.append(float(l["loss"]))
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)), losses
    changed = sum(int(not torch.equal(before[n], p)) for n, p in tr.nets.named_parameters())
    assert changed > 0.8 * len(before)


@pytest.mark.parametrize("name", ["mono", "stereo", "stereo_only", "no_ssim", "avg_reprojection", "no_automask",
                                  "predictive_mask", "v1_multiscale", "posecnn", "mono_nchw", "amp_bf16"])
def test_losses_match_oracle_on_same_outputs(name):
    """compute_losses (fused HIP) vs the oracle on identical network outputs + noise."""
    from oracle.md2_oracle import HotPathOptions, hot_path
    tr, batch = make(name)
    gen = torch.Generator().manual_seed(5)
    noise = {s: torch.randn(*tr.hot.noise_shape(s), generator=gen) for s in range(4)}
    tr.noise_override = {s: n.cuda() for s, n in noise.items()}
    with torch.no_grad():
        outputs = tr.nets(tr, batch)
        losses = tr.compute_losses(batch, outputs)
    o = tr.opt
    opt = HotPathOptions(height=H, width=W, frame_ids=o.frame_ids, v1_multiscale=o.v1_multiscale,
                         no_ssim=o.no_ssim, avg_reprojection=o.avg_reprojection,
                         disable_automasking=o.disable_automasking, predictive_mask=o.predictive_mask)
    cpu = {k: v.cpu() for k, v in batch.items()}
    disps = {s: outputs[("disp", s)].float().cpu() for s in range(4)}
    masks = {s: outputs["predictive_mask"][("disp", s)].cpu() for s in range(4)} if o.predictive_mask else None
    if o.pose_model_type == "posecnn":
        T = tr._stacked_T(batch, outputs).cpu()
        refs = []
        for s in range(4):   # per-scale T: run the oracle once per scale with that scale's T
            camT = {f: T[s, i] for i, f in enumerate(tr.src_frames)}
            ref, _ = hot_path(opt, disps, cpu, camT, noise=noise, keep_images=False, masks=masks)
            refs.append(float(ref[f"loss/{s}"]))
        got = [float(losses[f"loss/{s}"]) for s in range(4)]
        assert max(abs(a - b) for a, b in zip(got, refs)) < 1e-5, (got, refs)
        return
    T = tr._stacked_T(batch, outputs).cpu()
    camT = {f: T[i] for i, f in enumerate(tr.src_frames)}
    ref, _ = hot_path(opt, disps, cpu, camT, noise=noise, keep_images=False, masks=masks)
    for s in range(4):
        assert abs(float(losses[f"loss/{s}"]) - float(ref[f"loss/{s}"])) < 1e-5
    assert abs(float(losses["loss"]) - float(ref["loss"])) < 1e-5


def test_generate_images_pred_materialises_reference_keys():
    tr, batch = make("mono")
    with torch.no_grad():
        outputs = tr.nets(tr, batch)
        tr.generate_images_pred(batch, outputs)
        tr.compute_losses(batch, outputs)
    for s in range(4):
        assert outputs[("depth", 0, s)].shape == (B, 1, H, W)
        assert outputs["identity_selection/{}".format(s)].shape == (B, H, W)
        for f in (-1, 1):
            assert outputs[("sample", f, s)].shape == (B, H, W, 2)
            assert outputs[("color", f, s)].shape == (B, 3, H, W)
            assert outputs[("color_identity", f, s)] is batch[("color", f, 0)]


def test_batched_pose_pairs_match_separate_calls():
    """One pose-encoder pass over both pairs (bn_groups) == one call per pair."""
    tr, batch = make("mono")
    tr.set_train()
    import copy
    nets_ref = copy.deepcopy(tr.models)
    out = tr.predict_poses(batch, None)
    tr.batch_pose_pairs = False
    ref = tr.predict_poses(batch, None, models=nets_ref)
    for f in (-1, 1):
        for key in ("axisangle", "translation", "cam_T_cam"):
            torch.testing.assert_close(out[(key, 0, f)], ref[(key, 0, f)], rtol=1e-4, atol=1e-6)
    for (n, a), (_, b) in zip(tr.models["pose_encoder"].named_buffers(), nets_ref["pose_encoder"].named_buffers()):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=n)
    loss = sum(out[("cam_T_cam", 0, f)].square().sum() for f in (-1, 1))
    loss_r = sum(ref[("cam_T_cam", 0, f)].square().sum() for f in (-1, 1))
    ps = list(tr.models["pose_encoder"].parameters()) + list(tr.models["pose"].parameters())
    pr = list(nets_ref["pose_encoder"].parameters()) + list(nets_ref["pose"].parameters())
    ga = torch.autograd.grad(loss, ps, allow_unused=True)
    gb = torch.autograd.grad(loss_r, pr, allow_unused=True)
    worst = max(float((a - b).norm() / (b.norm() + 1e-12)) for a, b in zip(ga, gb) if b is not None)
    assert worst < 1e-3, worst


def test_checkpoint_roundtrip(tmp_path):
    tr, batch = make("mono", log_dir=str(tmp_path))
    tr.train_step(batch)
    folder = tr.save_model()
    assert sorted(os.listdir(folder)) == ["adam.pth", "depth.pth", "encoder.pth", "pose.pth", "pose_encoder.pth"]
    enc = torch.load(os.path.join(folder, "encoder.pth"), weights_only=True)
    assert enc["height"] == H and enc["width"] == W and "encoder.conv1.weight" in enc
    assert int(enc["encoder.bn1.num_batches_tracked"]) == 1   # folded BN counter written back
    penc = torch.load(os.path.join(folder, "pose_encoder.pth"), weights_only=True)
    assert int(penc["encoder.bn1.num_batches_tracked"]) == 2   # one pose-encoder call per frame pair
    tr2, _ = make("mono", log_dir=str(tmp_path), load_weights_folder=folder)
    for (n, p), (n2, p2) in zip(tr.nets.named_parameters(), tr2.nets.named_parameters()):
        assert n == n2 and torch.equal(p, p2)


def test_plane_bank_step_matches_per_call_splits(monkeypatch):
    """Three training steps with the conv weights split once per step (conv_ops.PlaneBank,
    one launch) update the networks bitwise like the per-convolution splits."""
    from monodepth2_amd import conv_ops
    monkeypatch.setattr(conv_ops, "AUTOTUNE", False)   # every eligible convolution on x6
    results = []
    for bank in (False, True):
        monkeypatch.setattr(conv_ops, "PLANE_BANK", bank)
        tr, batch = make("mono")
        losses = [float(tr.train_step(batch)[1]["loss"]) for _ in range(3)]
        torch.cuda.synchronize()
        results.append((losses, [p.detach().clone() for p in tr.nets.parameters()]))
    assert results[0][0] == results[1][0], (results[0][0], results[1][0])
    assert all(torch.equal(a, b) for a, b in zip(results[0][1], results[1][1]))
    assert conv_ops.plane_bank().entries, "the bank saw no x6 convolution"


def test_hip_graph_replay_matches_eager_step():
    """A replay of the captured step (networks on two streams, fused hot path,
    backward, capturable fused Adam) computes what the same step does eagerly from
    the same state: losses and updated parameters."""
    tr, batch = make("mono", hip_graph=True)
    tr.train_step(batch)                       # capture (+ warm-up steps) and one replay
    tr.train_step(batch)
    torch.cuda.synchronize()
    opt_state = [(p, {k: v for k, v in st.items()}) for p, st in tr.model_optimizer.state.items()]

    def snapshot():
        return ([p.detach().clone() for p in tr.nets.parameters()],
                [b.detach().clone() for b in tr.nets.buffers()],
                [{k: v.detach().clone() for k, v in st.items()} for _, st in opt_state],
                tr.seed_tensor.clone())

    def restore(snap):
        ps, bs, sts, seed = snap
        with torch.no_grad():
            for p, v in zip(tr.nets.parameters(), ps):
                p.copy_(v)
            for b, v in zip(tr.nets.buffers(), bs):
                b.copy_(v)
            for (_, st), saved in zip(opt_state, sts):
                for k, v in saved.items():
                    st[k].copy_(v)
            tr.seed_tensor.copy_(seed)

    snap = snapshot()
    _, lg = tr.train_step(batch)               # replay
    torch.cuda.synchronize()
    loss_graph = float(lg["loss"])
    params_graph = [p.detach().clone() for p in tr.nets.parameters()]
    restore(snap)
    _, le = tr.eager_step(tr.static_inputs)    # the same step, eagerly (on the capture's stream)
    torch.cuda.synchronize()
    assert abs(loss_graph - float(le["loss"])) < 1e-6, (loss_graph, float(le["loss"]))
    worst = max(float((a - b).abs().max()) for a, b in zip(params_graph, tr.nets.parameters()))
    assert worst < 1e-6, worst


def test_hip_graph_flat_sync_step_replays_eager_bitwise():
    """The multi-GPU graph path on one GPU: --grad_sync flat at world size 1 builds
    FlatGradSync's buckets (the collective itself is skipped at world size 1), so the
    captured step holds the per-parameter stream bookkeeping, the communication
    stream's waits on the producing streams (pose network on its own stream), the
    bucket copies and the join back.  A replay must equal the same step run eagerly
    from the same state, bit for bit, and every gradient must be its bucket view."""
    import warnings
    tr, batch = make("mono", hip_graph=True, grad_sync="flat")
    fs = tr.flat_sync
    assert fs is not None and fs.overlap and fs.comm is not None and len(fs.buckets) >= 1
    assert tr._pose_stream is not None
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        tr.train_step(batch)                       # capture (+ warm-up steps) and one replay
        tr.train_step(batch)
        for plist, views in zip(fs.buckets, fs.views):
            for p, v in zip(plist, views):
                assert p.grad is not None and p.grad.data_ptr() == v.data_ptr()
        loss_g, loss_e, worst, delta = _replay_vs_eager(tr, batch)
    # every accumulation on the stream its AccumulateGrad node was created on
    assert not [w for w in caught if "AccumulateGrad" in str(w.message)], [str(w.message) for w in caught]
    assert delta > 0
    assert loss_g == loss_e and worst == 0.0, (loss_g, loss_e, worst)


def _graph_state(tr):
    return ([p.detach().clone() for p in tr.nets.parameters()],
            [b.detach().clone() for b in tr.nets.buffers()])


def test_hip_graph_first_step_is_one_step():
    """The capture's warm-up steps leave no trace: after the first hip_graph
    train_step (warm-up + capture + one replay) the parameters, BatchNorm buffers and
    Adam state are those of ONE eager step from the same initial state (Adam step 1,
    not 4)."""
    tr, batch = make("mono", hip_graph=True)
    params0, bufs0 = _graph_state(tr)
    _, lg = tr.train_step(batch)
    torch.cuda.synchronize()
    loss_graph = float(lg["loss"])
    params_g, bufs_g = _graph_state(tr)
    steps = {float(st["step"]) for st in tr.model_optimizer.state.values()}
    assert steps == {1.0}, steps
    # the same first step eagerly, from the same initial state and zero Adam state
    with torch.no_grad():
        for p, v in zip(tr.nets.parameters(), params0):
            p.copy_(v)
        for b, v in zip(tr.nets.buffers(), bufs0):
            b.copy_(v)
        for st in tr.model_optimizer.state.values():
            for v in st.values():
                if torch.is_tensor(v):
                    v.zero_()
        tr.seed_tensor.zero_()
    _, le = tr.eager_step(tr.static_inputs)
    torch.cuda.synchronize()
    assert abs(loss_graph - float(le["loss"])) < 1e-6, (loss_graph, float(le["loss"]))
    for a, b in zip(params_g, tr.nets.parameters()):
        assert float((a - b).abs().max()) < 1e-6
    for a, b in zip(bufs_g, tr.nets.buffers()):
        assert float((a - b).abs().max()) < 1e-6


def test_hip_graph_replay_sees_lr_schedule():
    """StepLR's decay (trainer.py:505, x0.1 every scheduler_step_size epochs) reaches
    the replayed Adam: the lr lives in a device tensor the scheduler fills in place.
    A replay after the decay equals the same step run eagerly at the decayed lr."""
    tr, batch = make("mono", hip_graph=True)
    tr.train_step(batch)
    tr.train_step(batch)
    lr0 = float(tr.model_optimizer.param_groups[0]["lr"])
    for _ in range(tr.opt.scheduler_step_size):
        tr.model_lr_scheduler.step()
    assert abs(float(tr.model_optimizer.param_groups[0]["lr"]) - 0.1 * lr0) < 1e-12
    torch.cuda.synchronize()
    opt_state = [{k: v.detach().clone() for k, v in st.items()} for st in tr.model_optimizer.state.values()]
    params0, bufs0 = _graph_state(tr)
    seed0 = tr.seed_tensor.clone()
    tr.train_step(batch)                        # replay at the decayed lr
    torch.cuda.synchronize()
    params_g, _ = _graph_state(tr)
    with torch.no_grad():
        for p, v in zip(tr.nets.parameters(), params0):
            p.copy_(v)
        for b, v in zip(tr.nets.buffers(), bufs0):
            b.copy_(v)
        for st, saved in zip(tr.model_optimizer.state.values(), opt_state):
            for k, v in saved.items():
                st[k].copy_(v)
        tr.seed_tensor.copy_(seed0)
    tr.eager_step(tr.static_inputs)
    torch.cuda.synchronize()
    delta = max(float((a - b).abs().max()) for a, b in zip(params_g, params0))
    worst = max(float((a - b).abs().max()) for a, b in zip(params_g, tr.nets.parameters()))
    assert delta > 0
    assert worst < 1e-3 * delta + 1e-9, (worst, delta)


def test_encoder_input_matches_eager():
    """ResnetEncoder.prepare (md2_encoder_input) == (cat(frames) - 0.45) / 0.225 in
    channels_last, bit for bit, for one frame and for batched frame pairs."""
    from monodepth2_amd.networks import ResnetEncoder
    enc = ResnetEncoder(18, False, num_input_images=2).cuda().to(memory_format=torch.channels_last)
    enc1 = ResnetEncoder(18, False).cuda().to(memory_format=torch.channels_last)
    g = torch.Generator(device="cuda").manual_seed(0)
    fr = [torch.rand(3, 3, 16, 24, device="cuda", generator=g) for _ in range(3)]
    pairs = [[fr[1], fr[0]], [fr[0], fr[2]]]
    x = enc.prepare(pairs)
    ref = (torch.cat([torch.cat(p, 1) for p in pairs], 0) - 0.45) / 0.225
    assert x.is_contiguous(memory_format=torch.channels_last) and x.shape == ref.shape
    assert torch.equal(x, ref)
    x1 = enc1.prepare(fr[2])
    assert torch.equal(x1, (fr[2] - 0.45) / 0.225) and x1.is_contiguous(memory_format=torch.channels_last)
    # H*W not a multiple of 4: the one-pixel-per-thread kernel
    fo = [torch.rand(2, 3, 15, 23, device="cuda", generator=g) for _ in range(2)]
    xo = enc.prepare([[fo[0], fo[1]]])
    assert torch.equal(xo, (torch.cat(fo, 1) - 0.45) / 0.225)


def _replay_vs_eager(tr, batch):
    """Snapshot the training state, replay the captured step, restore, run the same
    step eagerly; returns (graph loss, eager loss, worst param diff, step delta)."""
    torch.cuda.synchronize()
    opt_state = [{k: v.detach().clone() for k, v in st.items()} for st in tr.model_optimizer.state.values()]
    params0, bufs0 = _graph_state(tr)
    seed0 = tr.seed_tensor.clone()
    _, lg = tr.train_step(batch)
    torch.cuda.synchronize()
    loss_g = float(lg["loss"])
    params_g, _ = _graph_state(tr)
    with torch.no_grad():
        for p, v in zip(tr.nets.parameters(), params0):
            p.copy_(v)
        for b, v in zip(tr.nets.buffers(), bufs0):
            b.copy_(v)
        for st, saved in zip(tr.model_optimizer.state.values(), opt_state):
            for k, v in saved.items():
                st[k].copy_(v)
        tr.seed_tensor.copy_(seed0)
    _, le = tr.eager_step(tr.static_inputs)
    torch.cuda.synchronize()
    delta = max(float((a - b).abs().max()) for a, b in zip(params_g, params0))
    worst = max(float((a - b).abs().max()) for a, b in zip(params_g, tr.nets.parameters()))
    return loss_g, float(le["loss"]), worst, delta


def _grads(tr):
    return [None if p.grad is None else p.grad.detach().clone() for p in tr.nets.parameters()]


def _rel_l2(a, b):
    num = sum(float((x - y).double().square().sum()) for x, y in zip(a, b) if x is not None and y is not None)
    den = sum(float(y.double().square().sum()) for x, y in zip(a, b) if x is not None and y is not None)
    return (num / den) ** 0.5


def _replay_eager_fp32(tr, batch):
    """From one snapshot of the training state: the captured step (replay), the same
    step eagerly, and the same step eagerly without autocast (fp32 networks); returns
    the three losses and the three steps' gradients."""
    torch.cuda.synchronize()
    opt_state = [{k: v.detach().clone() for k, v in st.items()} for st in tr.model_optimizer.state.values()]
    params0, bufs0 = _graph_state(tr)
    seed0 = tr.seed_tensor.clone()

    def restore():
        with torch.no_grad():
            for p, v in zip(tr.nets.parameters(), params0):
                p.copy_(v)
            for b, v in zip(tr.nets.buffers(), bufs0):
                b.copy_(v)
            for st, saved in zip(tr.model_optimizer.state.values(), opt_state):
                for k, v in saved.items():
                    st[k].copy_(v)
            tr.seed_tensor.copy_(seed0)

    _, lg = tr.train_step(batch)
    torch.cuda.synchronize()
    out = [(float(lg["loss"]), _grads(tr))]
    for amp in ("bf16", "none"):
        restore()
        tr.opt.amp = amp
        _, le = tr.eager_step(tr.static_inputs)
        torch.cuda.synchronize()
        out.append((float(le["loss"]), _grads(tr)))
    tr.opt.amp = "bf16"
    return out


@pytest.mark.parametrize("Bf", [2, 32])
def test_hip_graph_bf16_full_resolution_step(Bf):
    """Config C5's step (BASELINE configs[4]: bf16 autocast on the networks, the
    photometric loss in fp32, the whole step captured in one hipGraph) at the full
    640x192 resolution, at B=2 and at C5's own 32 images per GPU, and the replay's loss
    equals the CPU oracle (reference formulation, trainer.py:341-496) on the replay's
    own network outputs within 1e-5.

    At both batches a replay equals the same step run eagerly from the same state, bit for
    bit (loss and every parameter after Adam): the autocast convolutions run on the
    deterministic bf16 GEMMs (conv_ops.conv2d_bf16, MD2_CONV_BF16 — round 5's MIOpen bf16
    weight gradients made two replays differ by ~5 % gradient rel-L2 at B=32, DESIGN.md
    §6).  At B=32 the bf16 step is also held against the same step run in fp32 from the
    same state: within bf16's own error (bar 0.1 over all parameters), losses within 1e-4."""
    from oracle.md2_oracle import HotPathOptions, hot_path
    from monodepth2_amd.trainer import Trainer
    Hf, Wf = 192, 640
    torch.set_num_threads(16)
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=Bf, height=Hf, width=Wf, weights_init="scratch", log_dir="/tmp/md2_test",
                                 frame_ids=[0, -1, 1], amp="bf16", hip_graph=True), device=torch.device("cuda", 0))
    batch = synthetic_batch(Bf, Hf, Wf, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
    gen = torch.Generator().manual_seed(7)
    noise = {s: torch.randn(*tr.hot.noise_shape(s), generator=gen) for s in range(4)}
    tr.noise_override = {s: n.cuda() for s, n in noise.items()}
    tr.train_step(batch)       # warm-up + capture + first replay
    tr.train_step(batch)
    if Bf == 32:   # first: the graph's gradient tensors are p.grad only until an eager step
        (loss_g, g_g), (loss_e, g_e), (loss_f, g_f) = _replay_eager_fp32(tr, batch)
        assert loss_g == loss_e, (loss_g, loss_e)
        assert abs(loss_g - loss_f) < 1e-4, (loss_g, loss_f)
        assert _rel_l2(g_g, g_e) == 0.0
        e_g = _rel_l2(g_g, g_f)
        assert e_g < 0.1, e_g
    loss_g, loss_e, worst, delta = _replay_vs_eager(tr, batch)
    assert loss_g == loss_e, (loss_g, loss_e)
    assert delta > 0 and worst == 0.0, (worst, delta)
    # the replay's own outputs through the oracle
    _, lg = tr.train_step(batch)
    torch.cuda.synchronize()
    out = tr.static_outputs
    disps = {s: out[("disp", s)].detach().float().cpu() for s in range(4)}
    T = tr._stacked_T(tr.static_inputs, out).detach().cpu()
    cpu = {k: v.cpu() for k, v in tr.static_inputs.items()}
    ref, _ = hot_path(HotPathOptions(height=Hf, width=Wf, frame_ids=[0, -1, 1]), disps, cpu,
                      {f: T[i] for i, f in enumerate(tr.src_frames)}, noise=noise, keep_images=False)
    assert abs(float(lg["loss"]) - float(ref["loss"])) < 1e-5, (float(lg["loss"]), float(ref["loss"]))


def test_hip_graph_resume_keeps_device_lr(tmp_path):
    """Resuming a hip_graph run from a checkpoint (trainer.py:605-630 load_model, incl.
    adam.pth): the optimizer keeps its capturable form (device lr, device steps), the
    saved adam.pth has the reference's plain layout (float lr, CPU step tensors), and
    after the capture StepLR's decay still reaches the replays."""
    tr, batch = make("mono", log_dir=str(tmp_path), hip_graph=True)
    tr.train_step(batch)
    tr.train_step(batch)
    folder = tr.save_model()
    sd = torch.load(os.path.join(folder, "adam.pth"), weights_only=True)
    assert all(isinstance(g["lr"], float) and not g["capturable"] for g in sd["param_groups"])
    # no tensor hyper-parameter (StepLR's initial_lr included): loadable without a GPU
    assert not any(torch.is_tensor(v) for g in sd["param_groups"] for v in g.values())
    torch.load(os.path.join(folder, "adam.pth"), weights_only=True, map_location="cpu")
    assert all(v["step"].device.type == "cpu" and float(v["step"]) == 2.0 for v in sd["state"].values())
    tr2, batch2 = make("mono", log_dir=str(tmp_path), hip_graph=True, load_weights_folder=folder)
    g = tr2.model_optimizer.param_groups[0]
    assert torch.is_tensor(g["lr"]) and g["lr"].is_cuda and g["capturable"]
    assert all(st["step"].is_cuda for st in tr2.model_optimizer.state.values())
    tr2.train_step(batch2)
    tr2.train_step(batch2)
    assert {float(st["step"]) for st in tr2.model_optimizer.state.values()} == {4.0}
    lr0 = float(g["lr"])
    for _ in range(tr2.opt.scheduler_step_size):
        tr2.model_lr_scheduler.step()
    assert abs(float(tr2.model_optimizer.param_groups[0]["lr"]) - 0.1 * lr0) < 1e-15
    loss_g, loss_e, worst, delta = _replay_vs_eager(tr2, batch2)
    assert abs(loss_g - loss_e) < 1e-6
    assert delta > 0 and worst < 1e-3 * delta + 1e-9, (worst, delta)


def test_resnet50_1024x320_losses_match_oracle():
    """Config C4's shape (BASELINE configs[3]: mono 1024x320, ResNet-50, 8 images per
    GPU): the trainer's fused losses on its own network outputs equal the oracle's
    (reference formulation, trainer.py:407-496) within 1e-5 per scale and total."""
    from oracle.md2_oracle import HotPathOptions, hot_path
    from monodepth2_amd.trainer import Trainer
    Hc, Wc, Bc = 320, 1024, 8
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=Bc, height=Hc, width=Wc, num_layers=50, weights_init="scratch",
                                 log_dir="/tmp/md2_test", frame_ids=[0, -1, 1]), device=torch.device("cuda", 0))
    batch = synthetic_batch(Bc, Hc, Wc, tr.opt.frame_ids, 4, seed=11, device="cuda", eight_bit=True)
    tr.train_step(batch)            # one real step first: the outputs below are a trained state's
    gen = torch.Generator().manual_seed(9)
    noise = {s: torch.randn(*tr.hot.noise_shape(s), generator=gen) for s in range(4)}
    tr.noise_override = {s: n.cuda() for s, n in noise.items()}
    with torch.no_grad():
        outputs = tr.nets(tr, batch)
        losses = tr.compute_losses(batch, outputs)
    T = tr._stacked_T(batch, outputs).cpu()
    ref, _ = hot_path(HotPathOptions(height=Hc, width=Wc, frame_ids=[0, -1, 1]),
                      {s: outputs[("disp", s)].cpu() for s in range(4)}, {k: v.cpu() for k, v in batch.items()},
                      {f: T[i] for i, f in enumerate(tr.src_frames)}, noise=noise, keep_images=False)
    for s in range(4):
        assert abs(float(losses[f"loss/{s}"]) - float(ref[f"loss/{s}"])) < 1e-5, s
    assert abs(float(losses["loss"]) - float(ref["loss"])) < 1e-5


def test_hip_graph_needs_the_pose_stream(monkeypatch):
    """A captured step with the pose network on the main stream (--pose_streams 0) is
    refused when the Trainer is built, before any capture (open bug: its replays produce non-finite gradients,
    DESIGN.md §6; tools/onestream_graph_check.py reproduces it)."""
    from monodepth2_amd.trainer import Trainer
    monkeypatch.delenv("MD2_ALLOW_ONESTREAM_GRAPH", raising=False)
    with pytest.raises(ValueError, match="pose_streams"):
        Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch", log_dir="/tmp/md2_test",
                                hip_graph=True, pose_streams=0), device=torch.device("cuda", 0))
