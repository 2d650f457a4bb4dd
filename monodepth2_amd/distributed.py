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


class GradStreams:
    """Which HIP stream produced each parameter's gradient this step (the trainer's
    pose network runs its backward on its own stream).  A post-accumulate-grad hook
    notes the current stream inside the hook — the autograd node's — per parameter.

    DDP's comm hook uses it: DDP copies a gradient that autograd handed over as a fresh
    tensor (zero_grad(set_to_none=True)) into its bucket in its own hook, on the
    producing stream, AFTER this hook ran — so an event recorded here would not cover
    that copy.  But a bucket's comm hook only fires once every copy of the bucket has
    been queued; waiting there for the whole queue of each other producing stream
    covers them (the bucket's last gradient is on the current stream, which the
    collective's stream follows anyway).  Buckets whose gradients all came from the
    current stream wait for nothing, so the depth network's buckets still go out while
    the pose stream is busy."""

    def __init__(self, params):
        self.stream_of = {}
        self.handles = []
        for p in params:
            if p.requires_grad:
                self.handles.append(p.register_post_accumulate_grad_hook(self._ready))

    def _ready(self, p):
        if p.is_cuda:
            self.stream_of[p] = torch.cuda.current_stream(p.device)

    def wait(self, params, stream):
        for s in {self.stream_of[p] for p in params if p in self.stream_of}:
            if s != stream:
                stream.wait_stream(s)


def _stream_synced_allreduce(state, bucket):
    """DDP comm hook: the bucket's all-reduce follows every stream that produced one of
    its gradients (GradStreams), then the default all-reduce (average)."""
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
    state["streams"].wait(bucket.parameters(), torch.cuda.current_stream())
    return default_hooks.allreduce_hook(state["group"], bucket)


def wrap_ddp(module: nn.Module, device: torch.device, streams=None):
    """DDP over the networks.  `streams`: every HIP stream the backward writes
    gradients on (more than one -> the per-bucket event comm hook above)."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    DDP._set_params_and_buffers_to_ignore_for_model(module, ignored_parameters(module))
    gs = None
    if streams and len(streams) > 1:
        # registered before DDP's own autograd hooks: a parameter's producing stream is
        # noted before DDP can find its bucket ready and call the comm hook
        gs = GradStreams(module.parameters())
    kw = dict(broadcast_buffers=False, bucket_cap_mb=BUCKET_CAP_MB, gradient_as_bucket_view=True)
    if device.type == "cuda":
        kw.update(device_ids=[device.index], output_device=device.index)
    ddp = DDP(module, **kw)
    if gs is not None:
        ddp.register_comm_hook({"group": None, "streams": gs}, _stream_synced_allreduce)
        ddp._md2_grad_streams = gs
    return ddp


def shard(batch: Dict, rank: int, world: int) -> Dict:
    """Contiguous B/world slice of every batched tensor of a reference-keyed batch."""
    out = {}
    for k, v in batch.items():
        if k == "stereo_T" or (isinstance(k, tuple) and k[0] in ("color", "color_aug", "K", "inv_K")):
            n = v.shape[0] // world
            out[k] = v[rank * n:(rank + 1) * n]
        elif k == "color_src8":   # (S, B, H, W): the batch is the second axis
            n = v.shape[1] // world
            out[k] = v[:, rank * n:(rank + 1) * n].contiguous()
        else:
            out[k] = v
    return out


class FlatGradSync:
    """Gradient averaging over flat buckets, graph-capturable, overlapped with the
    backward.

    Parameters are bucketed in reverse registration order (the order the backward
    finishes them, as DDP).  `zero()` drops the gradients (autograd then hands each
    producer's output over instead of adding it into a zeroed buffer); a post-
    accumulate-grad hook per parameter notes the gradient and the stream it was
    produced on, and when a bucket's last gradient is final the bucket goes out (as
    soon as every bucket before it has: the collectives keep one order on every rank):
    the communication stream waits for the producing streams, copies the
    gradients into the flat buffer (one multi-tensor copy), and all-reduces it
    (ReduceOp.AVG on RCCL) — while the backward of the earlier layers continues.
    `sync()` sends any bucket still pending (parameters that got no gradient this step
    count as zero), makes the current stream wait for the communication stream, and
    points every `.grad` at its averaged view.  All of it is stream work ordered by
    events, so it can sit inside a captured hipGraph of the whole training step.
    Parameters that never get a gradient (the encoders' fc heads) are left out.
    `overlap=False`: the round-2 form (views of pre-zeroed buckets, one all-reduce per
    bucket after the backward), kept for comparison.

    The send order is calibrated on the first step at world > 1 (see `order` below):
    that step sends every bucket from sync(), after the backward, so it has no overlap.
    `recalibrate()` starts that over (the Trainer calls it before every capture's
    warm-up, so a re-capture or a changed stream layout measures its own order)."""

    def __init__(self, named_params, world: int, group=None, bucket_cap_mb: int = BUCKET_CAP_MB,
                 overlap: bool = True):
        self.world, self.group, self.overlap = world, group, overlap
        params = [(n, p) for n, p in named_params if p.requires_grad and not (
            n.endswith("encoder.fc.weight") or n.endswith("encoder.fc.bias"))]
        if overlap:
            params = params[::-1]
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
        self.flat, self.views = [], []
        self.where = {}
        for bi, plist in enumerate(self.buckets):
            buf = torch.zeros(sum(p.numel() for p in plist), dtype=torch.float32, device=plist[0].device)
            views, off = [], 0
            for p in plist:
                # the view keeps the parameter's strides (channels_last conv weights): the
                # gradient layout contract of autograd and the fused Adam kernel
                views.append(buf[off:off + p.numel()].as_strided(p.size(), p.stride()))
                self.where[p] = (bi, len(views) - 1)
                off += p.numel()
            self.flat.append(buf)
            self.views.append(views)
        if not overlap:
            for plist, views in zip(self.buckets, self.views):
                for p, v in zip(plist, views):
                    p.grad = v
            return
        cuda = self.flat and self.flat[0].is_cuda
        self.comm = torch.cuda.Stream(self.flat[0].device) if cuda else None
        self.pending = [dict() for _ in self.buckets]   # bucket -> {param: (grad, stream)}
        self.sent = [False] * len(self.buckets)
        self.next_send = 0   # position in self.order (see _ready)
        # send order: index order until calibrated.  At world > 1 the first step sends
        # every bucket from sync(), in index order, and notes the order the buckets
        # completed in; rank 0's order is broadcast once there (every rank present, no
        # backward running, not capturing) and every later step sends in it — a bucket
        # waits only for the buckets that finished before it on rank 0, not for every
        # lower index (the pose network's buckets no longer wait behind the depth
        # network's, nor the reverse)
        self.order = list(range(len(self.buckets)))
        self.calibrated = world <= 1
        self.finished = []
        self.handles = [p.register_post_accumulate_grad_hook(self._ready) for plist in self.buckets for p in plist]
        self.works = []

    def recalibrate(self):
        """Forget the adopted send order: the next step (at world > 1) sends in index
        order from sync() and measures the finish order again."""
        if self.overlap:
            self.order = list(range(len(self.buckets)))
            self.calibrated = self.world <= 1
            self.finished = []

    def zero(self):
        if not self.overlap:
            for buf in self.flat:
                buf.zero_()
            return
        for plist in self.buckets:
            for p in plist:
                p.grad = None
        self.pending = [dict() for _ in self.buckets]
        self.sent = [False] * len(self.buckets)
        self.next_send = 0
        self.works = []
        self.finished = []

    def _ready(self, p):
        bi, _ = self.where[p]
        if self.sent[bi]:
            return
        stream = torch.cuda.current_stream(p.device) if p.is_cuda else None
        self.pending[bi][p] = (p.grad, stream)
        if not self.calibrated:   # the calibration step: note the finish order, send from sync()
            if len(self.pending[bi]) == len(self.buckets[bi]):
                self.finished.append(bi)
            return
        # RCCL needs the same collective order on every rank, and autograd's hook order
        # need not be the same everywhere (a parameter without a gradient, another
        # stream finishing first): a complete bucket waits until every bucket before it
        # in self.order has gone out, as DDP's reducer launches its buckets in one order
        while self.next_send < len(self.order):
            b = self.order[self.next_send]
            if len(self.pending[b]) != len(self.buckets[b]):
                break
            self._send(b)
            self.next_send += 1

    def _send(self, bi):
        self.sent[bi] = True
        got = self.pending[bi]
        views = [v for p, v in zip(self.buckets[bi], self.views[bi]) if p in got]
        grads = [got[p][0] for p in self.buckets[bi] if p in got]
        missing = [v for p, v in zip(self.buckets[bi], self.views[bi]) if p not in got]
        buf = self.flat[bi]
        if self.comm is not None:
            for stream in {s for _, s in got.values() if s is not None}:
                self.comm.wait_stream(stream)
            with torch.cuda.stream(self.comm):
                self._fill(views, grads, missing)
                for g in grads:   # the producers' buffers stay alive until the copy ran
                    g.record_stream(self.comm)
                if self.world > 1:
                    dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group)
        else:
            self._fill(views, grads, missing)
            if self.world > 1:
                self.works.append(dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group, async_op=True))

    def _calibrate(self):
        """Rank 0's bucket finish order of this step (buckets that never completed
        follow in index order), adopted by every rank: one broadcast, here in sync()."""
        if self.flat and self.flat[0].is_cuda and torch.cuda.is_current_stream_capturing():
            return   # not inside a capture: keep index order, try again on an eager step
        seen = set(self.finished)
        mine = list(self.finished) + [b for b in range(len(self.buckets)) if b not in seen]
        box = [mine]
        dist.broadcast_object_list(box, src=0, group=self.group)
        self.order = [int(b) for b in box[0]]
        self.calibrated = True

    @staticmethod
    def _fill(views, grads, missing):
        if views:
            torch._foreach_copy_(views, grads)
        for v in missing:   # no gradient this step: it counts as zero, like a zeroed bucket
            v.zero_()

    def sync(self):
        if not self.overlap:
            if self.world <= 1:
                return
            for buf in self.flat:
                dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group)
            return
        for i in range(self.next_send, len(self.order)):   # the rest, in send order
            self._send(self.order[i])
        self.next_send = len(self.order)
        if not self.calibrated:
            self._calibrate()
        if self.comm is not None:
            torch.cuda.current_stream(self.flat[0].device).wait_stream(self.comm)
        for w in self.works:   # CPU (gloo): the asynchronous all-reduces
            w.wait()
        for plist, views in zip(self.buckets, self.views):
            for p, v in zip(plist, views):
                p.grad = v

