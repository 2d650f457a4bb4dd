"""Data parallelism on CPU with gloo, world size 2 (the GPU path uses RCCL).

Each rank runs the real depth/pose networks on its own batch shard with the oracle
hot-path loss (the HIP kernels need a GPU; the gradient-averaging logic under test
does not depend on the loss implementation).  After the gradient sync every rank
must hold the average of the per-shard gradients computed single-process, for both
sync strategies: DDP (eager steps) and FlatGradSync (graph-capturable buckets).
The classifier heads encoder.fc.* must be excluded from the sync.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from monodepth2_amd import networks
from monodepth2_amd.data import synthetic_batch
from monodepth2_amd.distributed import FlatGradSync, ignored_parameters, shard, wrap_ddp
from monodepth2_amd.layers import transformation_from_parameters

H, W, B_PER_RANK = 64, 64, 2
FRAMES = [0, -1, 1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Nets(torch.nn.Module):
    """Depth + pose networks behind one forward (as Trainer's _Networks), so DDP's
    forward pre-hooks run."""

    def __init__(self):
        super().__init__()
        enc = networks.ResnetEncoder(18, False)
        self.models = torch.nn.ModuleDict({
            "encoder": enc,
            "depth": networks.DepthDecoder(enc.num_ch_enc, range(4)),
            "pose_encoder": networks.ResnetEncoder(18, False, num_input_images=2),
        })
        self.models["pose"] = networks.PoseDecoder(self.models["pose_encoder"].num_ch_enc, 1, 2)

    def forward(self, inputs):
        m = self.models
        outputs = m["depth"](m["encoder"](inputs[("color_aug", 0, 0)]))
        for f in FRAMES[1:]:
            pair = [inputs[("color_aug", f, 0)], inputs[("color_aug", 0, 0)]] if f < 0 else \
                [inputs[("color_aug", 0, 0)], inputs[("color_aug", f, 0)]]
            a, t = m["pose"]([m["pose_encoder"](torch.cat(pair, 1))])
            outputs[("cam_T_cam", 0, f)] = transformation_from_parameters(a[:, 0], t[:, 0], invert=(f < 0))
        return outputs


def build_nets(seed=0):
    torch.manual_seed(seed)
    return Nets()


def loss_fn(nets, inputs):
    from oracle.md2_oracle import HotPathOptions, hot_path
    outputs = nets(inputs)
    camT = {f: outputs[("cam_T_cam", 0, f)] for f in FRAMES[1:]}
    gen = torch.Generator().manual_seed(99)
    noise = {s: torch.randn(inputs[("color", 0, 0)].shape[0], 2, H, W, generator=gen) for s in range(4)}
    losses, _ = hot_path(HotPathOptions(height=H, width=W, frame_ids=FRAMES),
                         {s: outputs[("disp", s)] for s in range(4)}, inputs, camT, noise=noise,
                         keep_images=False)
    return losses["loss"]


def full_batch():
    return synthetic_batch(2 * B_PER_RANK, H, W, FRAMES, 4, seed=7)


def _worker(rank, world, port, mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nets = build_nets()
    inputs = shard(full_batch(), rank, world)
    if mode == "ddp":
        model = wrap_ddp(nets, torch.device("cpu"))
        loss = loss_fn(model, inputs)
        loss.backward()
    else:
        # "flat": buckets sent from the backward's hooks as they complete (overlapped);
        # "flat_post": the round-2 form (zeroed buckets, all-reduce after the backward)
        sync = FlatGradSync(nets.named_parameters(), world, overlap=(mode == "flat"))
        for _ in range(2):   # a second step re-arms the hooks and buckets
            sync.zero()
            loss = loss_fn(nets, inputs)
            loss.backward()
            sync.sync()
    grads = {n: (p.grad.clone() if p.grad is not None else None) for n, p in nets.named_parameters()}
    torch.save(grads, os.path.join(out_dir, f"{mode}_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _reference_grads():
    """Average of the per-shard gradients, computed in one process."""
    torch.set_num_threads(4)
    batch = full_batch()
    acc = None
    for r in range(2):
        nets = build_nets()
        loss_fn(nets, shard(batch, r, 2)).backward()
        g = {n: p.grad.clone() for n, p in nets.named_parameters() if p.grad is not None}
        acc = g if acc is None else {n: acc[n] + g[n] for n in acc}
    return {n: v / 2 for n, v in acc.items()}


@pytest.fixture(scope="module")
def ref_grads():
    return _reference_grads()


@pytest.mark.parametrize("mode", ["ddp", "flat", "flat_post"])
def test_gradient_average_matches_single_process(mode, ref_grads, tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, mode, str(tmp_path)), nprocs=2, join=True)
    g0 = torch.load(os.path.join(tmp_path, f"{mode}_0.pt"), weights_only=True)
    g1 = torch.load(os.path.join(tmp_path, f"{mode}_1.pt"), weights_only=True)
    ignored = set(ignored_parameters(build_nets()))
    assert ignored and all(".encoder.fc." in n for n in ignored)
    checked = 0
    for n, ref in ref_grads.items():
        assert n not in ignored
        a, b = g0[n], g1[n]
        assert torch.equal(a, b), f"ranks disagree on {n}"
        torch.testing.assert_close(a, ref, rtol=1e-4, atol=1e-7)
        checked += 1
    assert checked > 100
    for n in ignored:
        assert g0[n] is None or float(g0[n].abs().sum()) == 0.0


def test_shard_slices_batched_tensors():
    batch = full_batch()
    s1 = shard(batch, 1, 2)
    assert torch.equal(s1[("color", 0, 0)], batch[("color", 0, 0)][B_PER_RANK:])
    assert torch.equal(s1[("K", 2)], batch[("K", 2)][B_PER_RANK:])
    assert s1[("color", -1, 3)].shape[0] == B_PER_RANK


def test_overlapped_buckets_equal_post_backward_sync(tmp_path):
    """The overlapped FlatGradSync (buckets all-reduced from the backward's hooks)
    gives bit for bit the gradients of the post-backward sync."""
    port = _free_port()
    mp.spawn(_worker, args=(2, port, "flat", str(tmp_path)), nprocs=2, join=True)
    port = _free_port()
    mp.spawn(_worker, args=(2, port, "flat_post", str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        a = torch.load(os.path.join(tmp_path, f"flat_{r}.pt"), weights_only=True)
        b = torch.load(os.path.join(tmp_path, f"flat_post_{r}.pt"), weights_only=True)
        for n in a:
            if a[n] is None or b[n] is None:
                assert (a[n] is None or float(a[n].abs().sum()) == 0) and (b[n] is None or float(b[n].abs().sum()) == 0)
                continue
            assert torch.equal(a[n], b[n]), n


def test_flat_sync_sends_buckets_in_index_order():
    """FlatGradSync hands buckets to the collective strictly in index order, whatever
    order the gradients finish in (RCCL needs one collective order on every rank;
    DDP's reducer launches its buckets in index order too).  Host logic only: the
    gradient hooks are fired by hand in a scrambled order."""
    params = [torch.nn.Parameter(torch.randn(4, 4)) for _ in range(6)]
    sync = FlatGradSync([(f"p{i}", p) for i, p in enumerate(params)], world=1, bucket_cap_mb=0)
    assert len(sync.buckets) == 6   # a zero cap: one parameter per bucket
    sent = []
    real_send = sync._send
    sync._send = lambda bi: (sent.append(bi), real_send(bi))
    sync.zero()
    order = [sync.buckets[i][0] for i in (3, 0, 5, 1, 2)]   # bucket 4 never gets a gradient
    for p in order:
        p.grad = torch.ones_like(p)
        sync._ready(p)
    assert sent == [0, 1, 2, 3]          # 3 waited for 1 and 2; 5 waits for 4
    sync.sync()
    assert sent == [0, 1, 2, 3, 4, 5]    # the rest, in order (4 counts as zero)
    b4 = sync.buckets[4][0]
    assert torch.equal(b4.grad, torch.zeros_like(b4)) and torch.equal(sync.buckets[5][0].grad, torch.ones(4, 4))


def _order_worker(rank, world, port, out_dir):
    """FlatGradSync at world 2 (gloo, CPU): the first step sends from sync() in index
    order and adopts rank 0's bucket finish order; later steps send in that order on
    every rank, whatever order their own hooks fire in, and average correctly."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    params = [torch.nn.Parameter(torch.zeros(4, 4)) for _ in range(6)]
    sync = FlatGradSync([(f"p{i}", p) for i, p in enumerate(params)], world=world, bucket_cap_mb=0)
    sent = []
    real_send = sync._send
    sync._send = lambda bi: (sent.append(bi), real_send(bi))
    fire = {0: (3, 0, 5, 1, 2), 1: (5, 4, 3, 2, 1, 0)}[rank]   # rank 0: bucket 4 gets no gradient
    res = {}
    for step in range(2):
        sync.zero()
        sent.clear()
        for b in fire:
            p = sync.buckets[b][0]
            p.grad = torch.full_like(p, float(rank + 1 + b))
            sync._ready(p)
        res[f"before_sync_{step}"] = list(sent)
        sync.sync()
        res[f"sent_{step}"] = list(sent)
        res[f"grads_{step}"] = [float(sync.buckets[b][0].grad[0, 0]) for b in range(6)]
    res["order"] = sync.order
    torch.save(res, os.path.join(out_dir, f"order_{rank}.pt"))
    dist.destroy_process_group()


def test_flat_sync_adopts_rank0_finish_order(tmp_path):
    port = _free_port()
    mp.spawn(_order_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (torch.load(os.path.join(tmp_path, f"order_{r}.pt"), weights_only=True) for r in range(2))
    for r in (r0, r1):
        assert r["before_sync_0"] == [] and r["sent_0"] == [0, 1, 2, 3, 4, 5]   # calibration step
        assert r["order"] == [3, 0, 5, 1, 2, 4]                               # rank 0's finish order
        assert r["sent_1"] == [3, 0, 5, 1, 2, 4]
    # rank 1's hooks fire 5, 4, 3, ...: nothing goes out before bucket 3 is complete there
    assert r1["before_sync_1"] == [3, 0, 5, 1, 2, 4][:len(r1["before_sync_1"])]
    for step in (0, 1):
        # mean of rank 0 (b + 1, or 0 for bucket 4 without a gradient) and rank 1 (b + 2)
        want = [((b + 1 if b != 4 else 0) + b + 2) / 2 for b in range(6)]
        assert r0[f"grads_{step}"] == want and r1[f"grads_{step}"] == want


def _autotune_worker(rank, world, port, out_dir):
    """The production conv-choice mechanism under data parallelism, host logic only (the
    candidates are stand-ins with rank-dependent timings: the ranks disagree).  Each
    rank autotunes inside its DDP forward and backward — rank 0 also runs an extra
    no_grad evaluation first that meets shapes in a different order (bench.py's
    rank-0-only parity check) — interleaved with DDP's bucket all-reduces; then
    agree_choices lines every rank up on rank 0's table at one known point."""
    import datetime
    from monodepth2_amd import conv_ops
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    # a collective inside the autotune would pair with the other rank's DDP all-reduce
    # or with a different shape's broadcast: fail fast instead of hanging
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    conv_ops.clear_choices()
    conv_ops._time_candidate = lambda fn: fn()          # a candidate returns (ms, repeatable)
    names = ["x6", "x6_256", "f32mfma", "miopen"]

    def cands(shape):
        # rank-dependent timings; on shape 1 the fastest candidate is not repeatable
        base = [1.0 + 0.1 * ((i + shape + rank) % 4) for i in range(4)]
        rep = [not (shape == 1 and i == int(min(range(3), key=lambda j: base[j]))) for i in range(4)]
        return [(lambda t=t, r=r: (t, r)) for t, r in zip(base, rep)]

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(8, 8)

        def forward(self, x, shapes):
            for sh in shapes:
                conv_ops._fastest("fwd", (sh,), cands(sh), names)
            return self.lin(x)

    torch.manual_seed(0)
    net = Net()
    ddp = torch.nn.parallel.DistributedDataParallel(net, bucket_cap_mb=1)

    class Hook(torch.autograd.Function):   # autotune calls inside the backward too
        @staticmethod
        def forward(ctx, y):
            return y

        @staticmethod
        def backward(ctx, g):
            for sh in (5, 6):
                conv_ops._fastest("wgrad", (sh,), cands(sh), names)
            return g

    if rank == 0:   # rank-0-only evaluation first, shapes in another order
        with torch.no_grad():
            net(torch.randn(2, 8), [3, 2, 9])
    for step in range(2):
        y = Hook.apply(ddp(torch.randn(4, 8), [0, 1, 2, 3, 4]))
        y.square().sum().backward()
        if step == 0:
            changed = conv_ops.agree_choices()
    table = {f"{k[0]} {k[1:]}": conv_ops._names[k][i] for k, i in conv_ops._choice.items()}
    # a shape rank 0 timed alone is pinned here to rank 0's choice for when it appears
    conv_ops._fastest("fwd", (9,), cands(9), names)
    table["after fwd (9,)"] = conv_ops._names[("fwd", 9)][conv_ops._choice[("fwd", 9)]]
    torch.save({"table": table, "changed": changed, "nondet": {str(k): v for k, v in conv_ops._nondet.items()}},
               os.path.join(out_dir, f"tune_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_conv_autotune_no_collective_then_rank0_table(tmp_path):
    port = _free_port()
    mp.spawn(_autotune_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(os.path.join(tmp_path, "tune_0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "tune_1.pt"), weights_only=True)
    assert r0["changed"] == 0 and r1["changed"] > 0          # rank 1 timed differently
    common = set(r0["table"]) & set(r1["table"])
    assert {"fwd (0,)", "fwd (4,)", "wgrad (5,)", "after fwd (9,)"} <= common
    for k in common:
        assert r0["table"][k] == r1["table"][k], k
    assert "fwd (9,)" not in r1["table"] or r1["table"]["fwd (9,)"] == r0["table"]["fwd (9,)"]
    # the fastest candidate of shape 1 returned different bits on a rerun: never kept
    for r in (r0, r1):
        assert any("1" in k for k in r["nondet"])
        assert r["table"]["fwd (1,)"] not in r["nondet"][next(k for k in r["nondet"] if "1" in k)]


def _union_worker(rank, world, port, out_dir):
    """agree_choices forms ONE table from every rank's choices: rank 0's choice where it
    has one, otherwise the lowest rank that met the shape.  A shape only rank 1 has met
    is pinned on rank 0 to rank 1's choice for when rank 0 meets it; a second agreement
    (run_epoch's) picks up shapes first met after the first one."""
    from monodepth2_amd import conv_ops
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    conv_ops.clear_choices()
    conv_ops._time_candidate = lambda fn: fn()
    names = ["x6", "x6_256", "f32mfma", "miopen"]

    def cands(shape):
        # rank- and shape-dependent fastest candidate: the ranks disagree on every shape
        return [(lambda i=i: (1.0 + 0.1 * ((i + shape + 2 * rank) % 3), True)) for i in range(4)]

    def pick(shape):
        return names[conv_ops._fastest("fwd", (shape,), cands(shape), names)]

    met = {0: [0, 1], 1: [1, 7]}[rank]
    own = {sh: pick(sh) for sh in met}
    res = {"own": own, "new_before": conv_ops.new_choices_since_agree()}
    res["changed1"] = conv_ops.agree_choices()
    res["new_after"] = conv_ops.new_choices_since_agree()
    res["seven"] = pick(7)                      # rank 0 meets rank 1's shape now: pinned
    later = 11 if rank == 1 else None           # a shape rank 1 alone meets after the agreement
    if later is not None:
        res["eleven_own"] = pick(later)
    res["changed2"] = conv_ops.agree_choices()
    res["eleven"] = pick(11)
    res["table"] = {str(k): conv_ops._names[k][i] for k, i in conv_ops._choice.items()}
    res["pinned"] = {str(k): v for k, v in conv_ops._pinned.items()}
    torch.save(res, os.path.join(out_dir, f"union_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_agree_choices_takes_the_union_of_every_ranks_shapes(tmp_path):
    port = _free_port()
    mp.spawn(_union_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (torch.load(os.path.join(tmp_path, f"union_{r}.pt"), weights_only=True) for r in range(2))
    assert r0["new_before"] == 2 and r1["new_before"] == 2
    assert r0["new_after"] == 0 and r1["new_after"] == 0
    assert r0["own"][1] != r1["own"][1]                    # the ranks timed shape 1 differently
    assert r0["pinned"] == r1["pinned"]                    # one table on every rank
    common = set(r0["table"]) & set(r1["table"])
    assert common == {"('fwd', 1)", "('fwd', 7)", "('fwd', 11)"}
    assert all(r0["table"][k] == r1["table"][k] for k in common)
    assert r1["pinned"]["('fwd', 0)"] == r0["own"][0]      # rank 0's shape pinned on rank 1
    assert r1["table"]["('fwd', 1)"] == r0["own"][1]       # rank 0's choice wins a shared shape
    assert r0["seven"] == r1["own"][7] == r1["seven"]      # rank 1's shape pinned on rank 0
    assert r0["eleven"] == r1["eleven_own"] == r1["eleven"]   # the second agreement
    assert r0["changed1"] == 0 and r1["changed1"] == 1


def _graph_guard_worker(rank, world, port, out_dir):
    """Trainer(hip_graph=True) at world size 2 on gloo: refused at construction with a
    message naming the backend, before any network is built or any step captured."""
    from monodepth2_amd.options import default_options
    from monodepth2_amd.trainer import Trainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    msg = None
    try:
        Trainer(default_options(batch_size=2, height=64, width=64, hip_graph=True, log_dir=str(out_dir)),
                device=torch.device("cpu"), rank=rank, world_size=world)
    except ValueError as e:
        msg = str(e)
    torch.save({"msg": msg}, os.path.join(out_dir, f"guard_{rank}.pt"))
    dist.destroy_process_group()


def test_hip_graph_on_gloo_is_refused_before_capture(tmp_path):
    port = _free_port()
    mp.spawn(_graph_guard_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        msg = torch.load(os.path.join(tmp_path, f"guard_{r}.pt"), weights_only=True)["msg"]
        assert msg is not None and "nccl" in msg and "gloo" in msg, msg
