"""Data parallelism through the real Trainer on the GPU: two ranks with the pose
network on its own HIP stream, so the gradient buckets receive gradients from two
streams.  After the synced backward every rank must hold the mean of the ranks'
local (no_sync) gradients.  Backends: gloo with both ranks on cuda:0 (the pool's
boxes have one GPU), and RCCL ("nccl") with one GPU per rank — skipped below two
GPUs; that is the path the 8-GPU run takes (comm stream, per-bucket stream waits,
RCCL's own stream)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port, backend):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # the local and the synced gradients come from two separate backward passes: the
    # convolutions MIOpen keeps must not use atomics (run-to-run rounding differences
    # would read as averaging errors); the autotune keeps no candidate whose repeated
    # outputs differ (conv_ops._time_candidate) either way
    torch.backends.cudnn.deterministic = True
    if backend == "nccl":
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
        return torch.device("cuda", rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return torch.device("cuda", 0)


def _first_step(tr, batch, rank):
    """The production convolution-choice path: rank 0 first runs a no_grad evaluation on
    its own (as bench.py's parity check does), then one real training step — the
    autotune times its candidates inside the forward and backward on each rank with no
    collective, and the Trainer lines every rank up on rank 0's table after the step
    (conv_ops.agree_choices).  Every rank then holds rank 0's choices, and no kept
    candidate failed its repeatability check."""
    from monodepth2_amd import conv_ops
    assert conv_ops.AUTOTUNE
    if rank == 0:
        with torch.no_grad():
            tr.nets(tr, batch)
    tr.train_step(batch)
    torch.cuda.synchronize()
    assert tr._choices_agreed
    mine = {k: conv_ops._names[k][i] for k, i in conv_ops._choice.items()}
    box = [mine]
    dist.broadcast_object_list(box, src=0)
    for k, v in box[0].items():
        assert k not in mine or mine[k] == v, (k, mine[k], v)
    for k, bad in conv_ops._nondet.items():   # evidence: never kept
        print(f"rank {rank}: non-repeatable candidates {bad} for {k}", flush=True)
        assert conv_ops._names[k][conv_ops._choice[k]] not in bad or not conv_ops.AUTOTUNE


def _rank_flat(rank, world, port, backend="gloo"):
    """FlatGradSync with the buckets sent from the backward's hooks on a communication
    stream (the graph-mode sync, run eagerly: gloo is not capturable): every rank's
    synced gradients equal the mean of the ranks' local gradients."""
    dev = _init(rank, world, port, backend)
    try:
        from monodepth2_amd.data import synthetic_batch
        from monodepth2_amd.options import default_options
        from monodepth2_amd.trainer import Trainer
        torch.manual_seed(0)
        tr = Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch", grad_sync="flat",
                                     log_dir="/tmp/md2_ddp_gpu"), device=dev, rank=rank, world_size=world)
        assert tr.ddp is None and tr.flat_sync is not None and tr.flat_sync.overlap
        tr.set_train()
        batch = synthetic_batch(2, 64, 128, tr.opt.frame_ids, 4, seed=10 + rank, device=dev)
        _first_step(tr, batch, rank)
        named = [(n, p) for n, p in tr.nets.named_parameters() if p.requires_grad and "fc." not in n]
        tr.flat_sync.zero()
        _, losses = tr.process_batch(batch)
        local = torch.autograd.grad(losses["loss"], [p for _, p in named], allow_unused=True)
        tr.flat_sync.zero()
        _, losses = tr.process_batch(batch)
        losses["loss"].backward()
        tr.flat_sync.sync()
        torch.cuda.synchronize()
        checked = 0
        for (n, p), lg in zip(named, local):
            if lg is None:
                continue
            mean = lg.clone()
            dist.all_reduce(mean)
            mean /= world
            err = float((p.grad - mean).norm() / (mean.norm() + 1e-12))
            assert err < 1e-5, (n, err)
            checked += 1
        assert checked > 100
    finally:
        dist.destroy_process_group()


def _rank(rank, world, port, backend="gloo"):
    dev = _init(rank, world, port, backend)
    try:
        from monodepth2_amd.data import synthetic_batch
        from monodepth2_amd.options import default_options
        from monodepth2_amd.trainer import Trainer
        torch.manual_seed(0)
        tr = Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch",
                                     log_dir="/tmp/md2_ddp_gpu"), device=dev, rank=rank, world_size=world)
        assert tr.ddp is not None and tr._pose_stream is not None
        tr.set_train()
        batch = synthetic_batch(2, 64, 128, tr.opt.frame_ids, 4, seed=10 + rank, device=dev)
        _first_step(tr, batch, rank)
        params = [p for p in tr.nets.parameters() if p.requires_grad]
        names = [n for n, p in tr.nets.named_parameters() if p.requires_grad]

        def grads():
            return [None if p.grad is None else p.grad.detach().clone() for p in params]

        tr.model_optimizer.zero_grad(set_to_none=True)
        with tr.ddp.no_sync():
            _, losses = tr.process_batch(batch)
            losses["loss"].backward()
        torch.cuda.synchronize()
        local = grads()
        tr.model_optimizer.zero_grad(set_to_none=True)
        _, losses = tr.process_batch(batch)
        losses["loss"].backward()
        torch.cuda.synchronize()
        synced = grads()
        checked = 0
        for n, lg, sg in zip(names, local, synced):
            if lg is None or "fc." in n:
                continue
            mean = lg.clone()
            dist.all_reduce(mean)
            mean /= world
            err = float((sg - mean).norm() / (mean.norm() + 1e-12))
            assert err < 1e-5, (n, err)
            checked += 1
        assert checked > 100
    finally:
        dist.destroy_process_group()


BACKENDS = ["gloo", pytest.param("nccl", marks=pytest.mark.skipif(
    torch.cuda.device_count() < 2, reason="RCCL needs one GPU per rank"))]


@pytest.mark.parametrize("backend", BACKENDS)
def test_ddp_with_pose_stream_averages_gradients(backend):
    mp.spawn(_rank, args=(2, _free_port(), backend), nprocs=2, join=True)


@pytest.mark.parametrize("backend", BACKENDS)
def test_flat_overlapped_sync_averages_gradients(backend):
    mp.spawn(_rank_flat, args=(2, _free_port(), backend), nprocs=2, join=True)
