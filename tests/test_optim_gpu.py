"""FusedAdam (one HIP launch per step, csrc/adam.hip) vs torch.optim.Adam on the same
parameters and gradients: updated parameters, moments and the state_dict layout
(reference checkpoints' adam.pth)."""
import copy

import pytest
import torch

from monodepth2_amd.optim import FusedAdam

pytestmark = pytest.mark.gpu


def _params(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    shapes = [(64, 3, 7, 7), (16, 32, 3, 3), (1, 16, 3, 3), (256,), (1,), (100003,), (12, 5)]
    ps = []
    for i, sh in enumerate(shapes):
        t = torch.randn(sh, device="cuda", generator=g)
        if len(sh) == 4 and i % 2 == 0:
            t = t.contiguous(memory_format=torch.channels_last)
        ps.append(torch.nn.Parameter(t))
    return ps


def test_fused_adam_matches_torch_adam():
    pa, pb = _params(0), _params(0)
    oa = FusedAdam(pa, lr=1e-3)
    ob = torch.optim.Adam(pb, lr=1e-3)   # the reference's optimizer (foreach on the GPU)
    g = torch.Generator(device="cuda").manual_seed(1)
    for step in range(4):
        for a, b in zip(pa, pb):
            gr = torch.randn(a.shape, device="cuda", generator=g)
            if a.dim() == 4 and a.is_contiguous(memory_format=torch.channels_last):
                gr = gr.contiguous(memory_format=torch.channels_last)   # grads follow their params
            a.grad = gr.clone()
            b.grad = gr.clone()
        oa.step()
        ob.step()
        if step == 1:   # the scheduler's lr edit reaches the kernel
            for o in (oa, ob):
                o.param_groups[0]["lr"] = 5e-4
    for a, b in zip(pa, pb):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
        sa, sb = oa.state[a], ob.state[b]
        # rounding-level differences only (torch's lerp form of the first-moment update)
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-9)
        assert float(sa["step"]) == float(sb["step"]) == 4.0
    assert oa.rebuilds == 1   # parameters and moments never moved


def test_fused_adam_state_dict_interchanges_with_torch_adam():
    pa, pb = _params(2), _params(2)
    ob = torch.optim.Adam(pb, lr=1e-3)
    for p in pb:
        p.grad = torch.ones_like(p)
    ob.step()
    oa = FusedAdam(pa, lr=1e-3)
    # a reference adam.pth into the fused optimizer (deep copy: as torch.save/load would,
    # so the two optimizers do not share moment buffers)
    oa.load_state_dict(copy.deepcopy(ob.state_dict()))
    for a, b in zip(pa, pb):
        with torch.no_grad():
            a.copy_(b)
        a.grad = torch.full_like(a, 0.5)
        b.grad = torch.full_like(b, 0.5)
    oa.step()
    ob.step()
    for a, b in zip(pa, pb):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    sd = oa.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"} and sd["state"][0]["step"].device.type == "cpu"


def test_fused_adam_shared_step_roundtrips_through_torch_adam():
    """The fast path keeps one step tensor for every state; its state_dict loaded into
    torch's Adam (or back into FusedAdam) still steps each parameter once."""
    pa, pb = _params(3), _params(3)
    oa = FusedAdam(pa, lr=1e-3)
    for _ in range(3):
        for p in pa:
            p.grad = torch.ones_like(p)
        oa.step()
    sd = oa.state_dict()
    assert all(float(s["step"]) == 3.0 for s in sd["state"].values())
    ob = torch.optim.Adam(pb, lr=1e-3)
    ob.load_state_dict(copy.deepcopy(sd))
    for p in pb:
        p.grad = torch.ones_like(p)
    ob.step()
    assert all(float(s["step"]) == 4.0 for s in ob.state.values())
    oc = FusedAdam(_params(3), lr=1e-3)
    oc.load_state_dict(sd)   # in memory: the step tensors arrive aliased
    steps = [s["step"] for s in oc.state.values()]
    assert len({id(t) for t in steps}) == len(steps)


def test_fused_adam_split_step_equals_single_launch():
    """The split capturable step (prepare_step at the start of a training step, then a
    tail of the parameters updated on another stream, FusedAdam.split) gives the
    parameters and moments of the one-launch capturable step bit for bit, including
    across an lr edit and on the first step (no table yet: prepare_step declines)."""
    pa, pb = _params(4), _params(4)
    oa = FusedAdam(pa, lr=1e-3, capturable=True)
    ob = FusedAdam(pb, lr=1e-3, capturable=True)
    side = torch.cuda.Stream()
    oa.split = (side, pa[3:])
    g = torch.Generator(device="cuda").manual_seed(5)
    prepared = []
    for step in range(5):
        prepared.append(oa.prepare_step())
        for a, b in zip(pa, pb):
            gr = torch.randn(a.shape, device="cuda", generator=g)
            if a.dim() == 4 and a.is_contiguous(memory_format=torch.channels_last):
                gr = gr.contiguous(memory_format=torch.channels_last)
            a.grad = gr.clone()
            b.grad = gr.clone()
        # the split's contract (md2_adam_apply_dev): the tail's update is ordered after
        # its parameters' gradients — in the Trainer they are produced on the side (pose)
        # stream itself; here they were written on the current stream, so the side stream
        # waits for it before the step enqueues the tail there
        side.wait_stream(torch.cuda.current_stream())
        oa.step()
        ob.step()
        if step == 2:
            for o in (oa, ob):
                o.param_groups[0]["lr"].fill_(5e-4)
    torch.cuda.synchronize()
    assert prepared == [False, True, True, True, True]
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
        assert torch.equal(oa.state[a]["exp_avg"], ob.state[b]["exp_avg"])
        assert torch.equal(oa.state[a]["exp_avg_sq"], ob.state[b]["exp_avg_sq"])
        assert float(oa.state[a]["step"]) == float(ob.state[b]["step"]) == 5.0
