"""Single-node data parallelism: one process per GPU, RCCL over xGMI.

The reference is single-GPU (README.md:147-155).  Every sample of the hot path is
independent, so the batch shards over ranks with no collective on the data path;
the only exchange is the gradient all-reduce (average) of the networks, done by
DDP in buckets overlapped with the backward pass.
On ROCm the "nccl" backend of torch.distributed is RCCL.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

# R18 depth+pose nets carry 26.8 M trainable fp32 parameters (107 MB of gradients);
# 64 MB buckets give two all-reduces per step, each big enough to use every xGMI link
BUCKET_CAP_MB = 64


def env_world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment.
    MD2_DEVICE_INDEX pins every rank to one device (one-GPU rehearsals with gloo)."""
    local = int(os.environ.get("LOCAL_RANK", 0))
    if "MD2_DEVICE_INDEX" in os.environ:
        local = int(os.environ["MD2_DEVICE_INDEX"])
    return int(os.environ.get("RANK", 0)), local, int(os.environ.get("WORLD_SIZE", 1))


def init_process_group(backend: str = None) -> Tuple[int, int, int]:
    """Initialise from the torch.distributed.run environment.  MD2_DIST_BACKEND
    overrides the backend (e.g. "gloo" to rehearse several ranks on one GPU)."""
    rank, local_rank, world = env_world()
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("MD2_DIST_BACKEND", backend)
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    return rank, local_rank, world


def ignored_parameters(module: nn.Module):
    """Parameters that never receive a gradient: the ImageNet classifier heads of the
    ResNet encoders (`encoder.fc.*`, kept only for checkpoint key parity)."""
    return [n for n, _ in module.named_parameters() if n.endswith("encoder.fc.weight")
            or n.endswith("encoder.fc.bias")]


def _stream_synced_allreduce(state, bucket):
    """DDP comm hook for a backward that runs on several HIP streams (the trainer's
    pose network has its own): a bucket's gradients may be written by any of them,
    and DDP's reducer only orders the all-reduce after the stream that completes the
    bucket.  Wait for every stream first, then the default mean all-reduce."""
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
    cur = torch.cuda.current_stream()
    for s in state["streams"]:
        if s.cuda_stream != cur.cuda_stream:
            cur.wait_stream(s)
    return default_hooks.allreduce_hook(state["group"], bucket)


def wrap_ddp(module: nn.Module, device: torch.device, streams=None):
    """DDP over the networks.  `streams`: every HIP stream the backward writes
    gradients on (more than one -> the synchronising comm hook above)."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    DDP._set_params_and_buffers_to_ignore_for_model(module, ignored_parameters(module))
    kw = dict(broadcast_buffers=False, bucket_cap_mb=BUCKET_CAP_MB, gradient_as_bucket_view=True)
    if device.type == "cuda":
        kw.update(device_ids=[device.index], output_device=device.index)
    ddp = DDP(module, **kw)
    if streams and len(streams) > 1:
        ddp.register_comm_hook({"group": None, "streams": list(streams)}, _stream_synced_allreduce)
    return ddp


def shard(batch: Dict, rank: int, world: int) -> Dict:
    """Contiguous B/world slice of every batched tensor of a reference-keyed batch."""
    out = {}
    for k, v in batch.items():
        if k == "stereo_T" or (isinstance(k, tuple) and k[0] in ("color", "color_aug", "K", "inv_K")):
            n = v.shape[0] // world
            out[k] = v[rank * n:(rank + 1) * n]
        else:
            out[k] = v
    return out


class FlatGradSync:
    """Gradient averaging over flat buckets, graph-capturable.

    Every trainable parameter's `.grad` is a view into one of a few flat fp32
    buckets (BUCKET_CAP_MB each).  After the backward pass `sync()` issues one
    all-reduce (ReduceOp.AVG on RCCL) per bucket; `zero()` clears the buckets
    with one memset each.  Unlike DDP's autograd hooks this is plain stream
    work, so it can sit inside a captured hipGraph of the whole training step.
    Parameters that never get a gradient (the encoders' fc heads) are left out.
    """

    def __init__(self, named_params, world: int, group=None, bucket_cap_mb: int = BUCKET_CAP_MB):
        self.world, self.group = world, group
        params = [(n, p) for n, p in named_params if p.requires_grad and not (
            n.endswith("encoder.fc.weight") or n.endswith("encoder.fc.bias"))]
        cap = bucket_cap_mb * (1 << 20) // 4
        self.buckets = []
        cur, size = [], 0
        for n, p in params:
            if cur and size + p.numel() > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self.flat = []
        for plist in self.buckets:
            buf = torch.zeros(sum(p.numel() for p in plist), dtype=torch.float32, device=plist[0].device)
            off = 0
            for p in plist:
                # the grad view keeps the parameter's strides (channels_last conv weights):
                # the gradient layout contract of autograd and the fused Adam kernel
                p.grad = buf[off:off + p.numel()].as_strided(p.size(), p.stride())
                off += p.numel()
            self.flat.append(buf)

    def zero(self):
        for buf in self.flat:
            buf.zero_()

    def sync(self):
        if self.world <= 1:
            return
        for buf in self.flat:
            dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group)
