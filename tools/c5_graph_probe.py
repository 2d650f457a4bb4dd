"""C5's captured step (bf16, B=32, 640x192): are the pose decoder's bias-add input
gradients the same on two replays from one state, and are the bias gradients?  A probe
Function on each bias-added map clones its incoming gradient inside the graph (the clone
is captured, its memory the graph's); after each replay the clones hold that replay's
values.  python tools/c5_graph_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from monodepth2_amd import conv_ops, decoder_ops  # noqa: E402
from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402

PROBES = {}
_count = {"i": 0}


class _Probe(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, name):
        ctx.name = name
        return z.view_as(z)

    @staticmethod
    def backward(ctx, g):
        PROBES[ctx.name] = g.detach().clone()
        s = g.float().sum((0, 2, 3))
        PROBES[ctx.name + " sum"] = s
        return g, None


_orig = decoder_ops.conv_bias_act


def probed(conv, x, relu):
    if not conv_ops._bf16_ok(x, conv.weight, conv.stride[0], conv.padding[0]):
        return _orig(conv, x, relu)
    name = "pose%d" % (_count["i"] % 4)
    _count["i"] += 1
    z = conv_ops.conv2d_bf16(x, conv.weight, conv.stride[0], conv.padding[0])
    PROBES[name + " conv out"] = z
    z = z + conv.bias.to(torch.bfloat16).view(1, -1, 1, 1)
    z = _Probe.apply(z, name)
    return F.relu(z) if relu else z


decoder_ops.conv_bias_act = probed


def main():
    Hf, Wf, B = 192, 640, 32
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=B, height=Hf, width=Wf, weights_init="scratch", log_dir="/tmp/md2_probe",
                                 frame_ids=[0, -1, 1], amp="bf16", hip_graph=True), device=torch.device("cuda", 0))
    batch = synthetic_batch(B, Hf, Wf, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
    gen = torch.Generator().manual_seed(7)
    tr.noise_override = {s: torch.randn(*tr.hot.noise_shape(s), generator=gen).cuda() for s in range(4)}
    tr.train_step(batch)
    tr.train_step(batch)
    torch.cuda.synchronize()
    names = [n for n, _ in tr.nets.named_parameters()]
    opt_state = [{k: v.detach().clone() for k, v in st.items()} for st in tr.model_optimizer.state.values()]
    p0 = [p.detach().clone() for p in tr.nets.parameters()]
    b0 = [b.detach().clone() for b in tr.nets.buffers()]
    seed0 = tr.seed_tensor.clone()
    runs = []
    for r in range(4):
        with torch.no_grad():
            for p, v in zip(tr.nets.parameters(), p0):
                p.copy_(v)
            for b, v in zip(tr.nets.buffers(), b0):
                b.copy_(v)
            for st, saved in zip(tr.model_optimizer.state.values(), opt_state):
                for k, v in saved.items():
                    st[k].copy_(v)
            tr.seed_tensor.copy_(seed0)
        tr.train_step(batch)
        torch.cuda.synchronize()
        snap = {k: v.detach().clone() for k, v in PROBES.items()}
        for n, p in tr.nets.named_parameters():
            if n.startswith("models.pose.") and p.grad is not None:
                snap["grad " + n] = p.grad.detach().clone()
        runs.append(snap)
    for r in range(1, len(runs)):
        print("== replay %d vs replay 0" % r)
        for k in sorted(runs[0]):
            a, b = runs[0][k], runs[r][k]
            same = torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                               b.view(torch.int16) if b.dtype == torch.bfloat16 else b)
            print("  %-40s %s%s" % (k, "same" if same else "DIFF",
                                    "" if same else "  max %.3e" % float((a.float() - b.float()).abs().max())))


if __name__ == "__main__":
    main()
