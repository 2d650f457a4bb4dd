"""Adam for the training step (trainer.py:102-104, 209) with the update in one HIP
launch (md2_adam_step, csrc/adam.hip).

`FusedAdam` IS a `torch.optim.Adam`: same constructor, param groups, lr scheduler
hooks and `state_dict()` layout (per parameter `step` (CPU scalar tensor),
`exp_avg`, `exp_avg_sq`), so reference checkpoints (`adam.pth`) load and save
unchanged.  Only `step()` differs: instead of torch's multi-tensor kernels it walks a
device table of <=CHUNK-element chunks (param, exp_avg, exp_avg_sq), built once (those
buffers do not move), with the step's gradient pointers as kernel arguments — one
launch per 256 parameters.  Anything the kernel does not cover (CPU tensors, non-fp32,
sparse grads, a grad whose strides differ from its parameter's, amsgrad, weight
decay, maximize, capturable) goes through torch's own Adam step.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

CHUNK = 1 << 16   # elements per table entry (one block)


class FusedAdam(torch.optim.Adam):
    """capturable=True: the hipGraph form (torch's `capturable` semantics) — the lr is
    a device fp64 tensor (StepLR fills it in place, so replays see the decay), the
    step counters are device tensors advanced by the kernel launch itself
    (md2_adam_step_dev), so the whole step can be captured and replayed."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, capturable: bool = False):
        params = list(params)
        if capturable and not torch.is_tensor(lr):
            first = params[0]["params"][0] if isinstance(params[0], dict) else params[0]
            lr = torch.tensor(float(lr), dtype=torch.float64, device=first.device)
        super().__init__(params, lr=lr, betas=betas, eps=eps, capturable=capturable)
        self.capturable = capturable
        self._hyper = None   # device scratch of the capturable launch (step size, sqrt(bc2))
        self._key = None
        self._table = None
        self._starts = None
        self._grads = None
        self._params = None   # the parameter list the table was built for
        self._step_t = None   # on the fast path every state's "step" is this one CPU tensor
        self.rebuilds = 0   # chunk-table uploads (a parameter or moment buffer moved)
        self._hyper_ev = None   # prepare_step: the step's bias-correction factors are on the device
        self.split = None       # (side stream, parameters): that tail of the parameters updates there

    def state_dict(self):
        """torch's layout, each parameter with its own step tensor (a reference Adam
        loading adam.pth increments them one by one).  The capturable form saves what a
        plain torch.optim.Adam saves (float lr, CPU step tensors, capturable False), so
        adam.pth stays interchangeable with the reference's."""
        sd = super().state_dict()
        if self._step_t is not None or self.capturable:
            sd["state"] = {k: ({**v, "step": v["step"].detach().clone().cpu()} if "step" in v else v)
                           for k, v in sd["state"].items()}
        if self.capturable:
            # every tensor hyper-parameter as a float: lr, and StepLR's initial_lr (a
            # cloned device fp64 tensor in torch 2.10) — adam.pth then holds no CUDA
            # tensor and loads on a CPU-only machine like the reference's
            sd["param_groups"] = [{**{k: (float(v) if torch.is_tensor(v) else v) for k, v in g.items()},
                                   "capturable": False, "fused": None}
                                  for g in sd["param_groups"]]
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._key = None   # new moment buffers: rebuild the table on the next step
        self._step_t = None
        if self.capturable:
            # torch takes the saved groups' hyper-parameters (a reference adam.pth has a
            # float lr and capturable False): back to the device lr and device steps
            for g in self.param_groups:
                dev = g["params"][0].device
                g["lr"] = torch.tensor(float(g["lr"]), dtype=torch.float64, device=dev)
                g["capturable"] = True
                g["fused"] = None
                for p in g["params"]:
                    st = self.state.get(p)
                    if st and torch.is_tensor(st.get("step")):
                        st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
        # a state_dict saved from the fast path carries one step tensor under every
        # parameter: give each state its own, as torch's Adam increments them one by one
        seen = set()
        for st in self.state.values():
            t = st.get("step")
            if t is None:
                continue
            if id(t) in seen:
                st["step"] = t.clone()
            else:
                seen.add(id(t))

    def _unshare_steps(self):
        """Before torch's own step (which increments each state's "step" in place):
        give every state its own step tensor again."""
        if self._step_t is None:
            return
        for st in self.state.values():   # every group (add_param_group may have run since)
            if st.get("step") is self._step_t:
                st["step"] = self._step_t.clone()
        self._step_t = None

    def _group_ok(self) -> bool:
        if len(self.param_groups) != 1:   # one lr / betas / eps per launch
            return False
        g = self.param_groups[0]
        if bool(g.get("capturable")) != self.capturable:
            return False
        if self.capturable and not (torch.is_tensor(g["lr"]) and g["lr"].dtype == torch.float64
                                    and g["lr"].is_cuda):
            return False
        return not (g["weight_decay"] != 0 or g["amsgrad"] or g["maximize"] or g.get("differentiable"))

    def _eligible(self) -> bool:
        if not self._group_ok():
            return False
        for p in self.param_groups[0]["params"]:
            if p.grad is None:
                continue
            if (not p.is_cuda or p.dtype != torch.float32 or p.grad.dtype != torch.float32 or p.grad.is_sparse
                    or p.grad.stride() != p.stride() or not _dense(p)):
                return False
        return True

    def _fast_ok(self, params) -> bool:
        """Per-step check once the table is built for exactly these parameters: the
        parameters' own properties (device, dtype, density) were checked at build time
        and cannot change without a new tensor (caught by the data_ptr comparison);
        only the gradients, new every step, are looked at."""
        if not self._group_ok() or len(params) != len(self._params):
            return False
        for p, q, k in zip(params, self._params, self._key):
            g = p.grad
            if (p is not q or p.data_ptr() != k[0] or g.dtype != torch.float32 or g.is_sparse
                    or g.stride() != p.stride()):
                return False
        return True

    def _state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = (torch.zeros((), dtype=torch.float32, device=p.device) if self.capturable
                          else torch.tensor(0.0))
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    def _build(self, params):
        rows, starts = [], [0]
        for k, p in enumerate(params):
            st = self.state[p]
            base = [p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()]
            n = p.numel()
            for off in range(0, n, CHUNK):
                rows.append([b + 4 * off for b in base] + [off, min(CHUNK, n - off), k])
            starts.append(len(rows))
        host = torch.from_numpy(np.asarray(rows, dtype=np.int64).reshape(-1)).pin_memory()
        self._table = torch.empty(host.numel(), dtype=torch.int64, device=params[0].device)
        self._table.copy_(host, non_blocking=True)
        self._starts = (ctypes.c_int * len(starts))(*starts)
        self._grads = (ctypes.c_void_p * len(params))()
        self.rebuilds += 1

    def prepare_step(self) -> bool:
        """Capturable form: advance the device step counter and form this step's bias
        corrections now (md2_adam_hyper, one thread), at the start of a training step, so
        that `step()` can update part of the parameters on another stream (`split`)
        without that stream waiting for this one's backward.  False (and nothing done)
        where the split step does not apply; then `step()` does it all."""
        if not (self.capturable and self._key is not None and self._step_t is not None and self._group_ok()):
            return False
        group = self.param_groups[0]
        dev = group["params"][0].device
        if self._hyper is None:
            self._hyper = torch.empty(2, dtype=torch.float32, device=dev)
        b1, b2 = group["betas"]
        _lib.check(_lib.lib().md2_adam_hyper(group["lr"].data_ptr(), float(b1), float(b2), self._step_t.data_ptr(),
                                             self._hyper.data_ptr(), _lib.stream(dev)), "md2_adam_hyper")
        self._hyper_ev = torch.cuda.Event()
        self._hyper_ev.record(torch.cuda.current_stream(dev))
        return True

    def _undo_prepare(self):
        """A prepared step that falls back to torch's Adam: its counter goes back (torch
        advances it itself)."""
        if self._hyper_ev is not None:
            self._hyper_ev = None
            self._step_t.sub_(1)

    def _step_split(self, params, group) -> bool:
        """The rest of a prepared capturable step: the parameters of `split` (a tail of
        this step's list) on the split's stream, the others here, both after the
        factors prepare_step formed; this stream then waits for the split's."""
        ev, self._hyper_ev = self._hyper_ev, None
        side, tail = self.split if self.split is not None else (None, ())
        ids = {id(p) for p in tail}
        k = len(params)
        while k > 0 and id(params[k - 1]) in ids:
            k -= 1
        if side is None or k == len(params) or any(id(p) in ids for p in params[:k]):
            k = len(params)   # no contiguous tail: everything here
        b1, b2 = group["betas"]
        L = _lib.lib()
        dev = params[0].device
        cur = torch.cuda.current_stream(dev)
        cur.wait_event(ev)
        if k < len(params):
            side.wait_event(ev)
            _lib.check(L.md2_adam_apply_dev(self._table.data_ptr(), self._starts, k, len(params), self._grads,
                                            float(b1), float(b2), float(group["eps"]), self._hyper.data_ptr(),
                                            ctypes.c_void_p(side.cuda_stream)), "md2_adam_apply_dev")
        _lib.check(L.md2_adam_apply_dev(self._table.data_ptr(), self._starts, 0, k, self._grads, float(b1),
                                        float(b2), float(group["eps"]), self._hyper.data_ptr(), _lib.stream(dev)),
                   "md2_adam_apply_dev")
        if k < len(params):
            cur.wait_stream(side)
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        group = self.param_groups[0]
        params = [p for p in group["params"] if p.grad is not None]
        fast = self._key is not None and self._fast_ok(params)
        if not fast and not self._eligible():
            self._undo_prepare()
            self._key = None
            self._unshare_steps()
            return super().step()
        if not params:
            return loss
        states = [self._state(p) for p in params]
        # the table holds parameters and moments, which do not move; gradients (new
        # buffers every step) travel as kernel arguments.  Moments only move through
        # load_state_dict (which drops the table) or a new state (a new parameter list).
        if not fast:
            key = tuple((p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel())
                        for p, st in zip(params, states))
            if key != self._key:
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("FusedAdam: the parameter set changed during hipGraph capture "
                                       "(run an eager step first)")
                # (re)validate what the kernel assumes, then upload the chunk table
                if (len({float(st["step"]) for st in states}) != 1
                        or any(st["exp_avg"].stride() != p.stride() or st["exp_avg_sq"].stride() != p.stride()
                               for p, st in zip(params, states))):
                    self._undo_prepare()
                    self._key = None
                    self._unshare_steps()
                    return super().step()   # mixed step counts / layouts (e.g. a loaded partial state)
                self._build(params)
                self._key = key
            self._params = list(params)
        # the step counters (CPU scalars, as torch's Adam keeps them; all equal here) are
        # one shared tensor: one increment per step instead of a foreach over every
        # parameter (~0.4 ms of host time per step)
        if self._step_t is None or any(st["step"] is not self._step_t for st in states):
            self._step_t = states[0]["step"].clone()
            for st in states:
                st["step"] = self._step_t
        if not fast:
            # a parameter without a gradient this step keeps its own counter (torch's
            # Adam leaves its step alone)
            # (a step prepared at its start has already advanced the shared counter:
            # such a parameter keeps the value from before this step)
            prepared = self.capturable and self._hyper_ev is not None
            live = {id(st) for st in states}
            for st in self.state.values():
                if id(st) not in live and st.get("step") is self._step_t:
                    st["step"] = self._step_t.clone().sub_(1) if prepared else self._step_t.clone()
        b1, b2 = group["betas"]
        for k, p in enumerate(params):
            self._grads[k] = p.grad.data_ptr()
        if self.capturable and self._hyper_ev is not None:
            if fast:   # the step prepared at its start (prepare_step): the update alone, split
                self._step_split(params, group)
                return loss
            self._hyper_ev = None   # the table changed: prepare_step already advanced the counter
            rc = _lib.lib().md2_adam_apply_dev(self._table.data_ptr(), self._starts, 0, len(params), self._grads,
                                               float(b1), float(b2), float(group["eps"]), self._hyper.data_ptr(),
                                               _lib.stream(params[0].device))
            _lib.check(rc, "md2_adam_apply_dev")
            return loss
        if self.capturable:
            # the kernel launch advances the device step counter itself
            if self._hyper is None:
                self._hyper = torch.empty(2, dtype=torch.float32, device=params[0].device)
            rc = _lib.lib().md2_adam_step_dev(self._table.data_ptr(), self._starts, len(params), self._grads,
                                              group["lr"].data_ptr(), float(b1), float(b2), float(group["eps"]),
                                              self._step_t.data_ptr(), self._hyper.data_ptr(),
                                              _lib.stream(params[0].device))
            _lib.check(rc, "md2_adam_step_dev")
            return loss
        self._step_t += 1
        step = int(self._step_t)
        lr = group["lr"]
        lr = float(lr) if not torch.is_tensor(lr) else float(lr.item())
        rc = _lib.lib().md2_adam_step(self._table.data_ptr(), self._starts, len(params), self._grads, lr,
                                      float(b1), float(b2), float(group["eps"]), step,
                                      _lib.stream(params[0].device))
        _lib.check(rc, "md2_adam_step")
        return loss


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: the storage span equals numel (any dim order)."""
    if t.numel() == 0:
        return True
    span = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()) if s > 1)
    return span == t.numel() and all(st >= 0 for st in t.stride())
