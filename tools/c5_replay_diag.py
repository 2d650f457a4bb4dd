"""Config C5's captured bf16 step at B=32 640x192: replay vs the same step run eagerly
from the same state (tests/test_trainer_gpu.py::test_hip_graph_bf16_full_resolution_step),
per parameter: the worst parameter difference after the step, against the step size,
and the gradients' difference, with Adam's normalised update |m/(sqrt(v)+eps)| at the
worst element (an element whose gradient is ~eps-sized moves by a whole step for a
rounding-level gradient change).  python tools/c5_replay_diag.py [--batch 32] [--fp32 0]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--amp", default="bf16")
    ap.add_argument("--deterministic", type=int, default=0, help="MIOpen deterministic algorithms only")
    ap.add_argument("--pose-streams", type=int, default=1, help="0: the pose network on the main stream")
    ap.add_argument("--first", default="graph", choices=["graph", "eager"], help="the first run of the step")
    ap.add_argument("--second", default="eager", choices=["eager", "graph", "fp32"],
                    help="what the replay is compared with: the eager step, or a second replay")
    a = ap.parse_args()
    torch.backends.cudnn.deterministic = bool(a.deterministic)
    Hf, Wf, B = 192, 640, a.batch
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=B, height=Hf, width=Wf, weights_init="scratch", log_dir="/tmp/md2_diag",
                                 frame_ids=[0, -1, 1], amp=a.amp, hip_graph=True,
                                 pose_streams=a.pose_streams), device=torch.device("cuda", 0))
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
    _, lg = tr.train_step(batch) if a.first == "graph" else tr.eager_step(tr.static_inputs)
    torch.cuda.synchronize()
    pg = [p.detach().clone() for p in tr.nets.parameters()]
    gg = [None if p.grad is None else p.grad.detach().clone() for p in tr.nets.parameters()]
    with torch.no_grad():
        for p, v in zip(tr.nets.parameters(), p0):
            p.copy_(v)
        for b, v in zip(tr.nets.buffers(), b0):
            b.copy_(v)
        for st, saved in zip(tr.model_optimizer.state.values(), opt_state):
            for k, v in saved.items():
                st[k].copy_(v)
        tr.seed_tensor.copy_(seed0)
    if a.second == "fp32":   # the same step's gradients without autocast: the accuracy reference
        tr.opt.amp = "none"
        _, le = tr.eager_step(tr.static_inputs)
    else:
        _, le = tr.eager_step(tr.static_inputs) if a.second == "eager" else tr.train_step(batch)
    torch.cuda.synchronize()
    ge = [None if p.grad is None else p.grad.detach().clone() for p in tr.nets.parameters()]
    print("loss graph %.9g eager %.9g" % (float(lg["loss"]), float(le["loss"])))
    rows = []
    st = list(tr.model_optimizer.state.values())
    pidx = {id(p): i for i, p in enumerate(tr.nets.parameters())}
    state_of = {}
    for grp in tr.model_optimizer.param_groups:
        for p in grp["params"]:
            state_of[pidx[id(p)]] = tr.model_optimizer.state.get(p)
    for i, n in enumerate(names):
        d = (pg[i] - tr.nets.get_parameter(n).detach()).abs()
        step = (pg[i] - p0[i]).abs().max()
        if gg[i] is None or ge[i] is None:
            continue
        gd = float((gg[i] - ge[i]).norm() / ge[i].norm().clamp_min(1e-30))
        k = int(d.flatten().argmax())
        s = state_of.get(i)
        upd = float("nan")
        if s is not None and "exp_avg" in s:
            m, v = s["exp_avg"].flatten()[k], s["exp_avg_sq"].flatten()[k]
            upd = float(m.abs() / (v.sqrt() + 1e-8))
        rows.append((float(d.max()), n, float(step), gd, float(ge[i].flatten()[k]), upd))
    rows.sort(reverse=True)
    for r in rows[:12]:
        print("worst %.3e  %-48s step %.3e  grad rel-L2 %.3e  grad@worst %.3e  |m|/(sqrt v+eps)@worst %.3f" % r)
    print("grad rel-L2 max over params: %.3e" % max(r[3] for r in rows))
    num = sum(float((g - e).double().square().sum()) for g, e in zip(gg, ge) if g is not None and e is not None)
    den = sum(float(e.double().square().sum()) for g, e in zip(gg, ge) if g is not None and e is not None)
    print("grad rel-L2 over all params: %.3e" % (num / den) ** 0.5)
    # every parameter whose gradient differs at all, in module order (the last one in
    # forward order sits closest to the op that differs), and the autotune's bf16 choices
    for i, n in enumerate(names):
        if gg[i] is not None and ge[i] is not None and not torch.equal(gg[i], ge[i]):
            print("differs %-48s rel-L2 %.3e  |first| %.3e |second| %.3e" % (
                n, float((gg[i] - ge[i]).norm() / ge[i].norm().clamp_min(1e-30)), float(gg[i].norm()),
                float(ge[i].norm())))
            dd = (gg[i] - ge[i]).flatten()
            nz = torch.nonzero(dd).flatten()
            print("   %d of %d elements differ; at %s: %s vs %s" % (
                nz.numel(), dd.numel(), nz[:6].tolist(), gg[i].flatten()[nz[:6]].tolist(),
                ge[i].flatten()[nz[:6]].tolist()))
            if gg[i].numel() <= 16:
                print("   graph", gg[i].flatten().tolist())
                print("   eager", ge[i].flatten().tolist())
    from monodepth2_amd import conv_ops
    for k, i in conv_ops._choice.items():
        if k in conv_ops._names and k[0].endswith("bf16"):
            print("choice", k, conv_ops._names[k][i], "nondet" if k in conv_ops._nondet else "")


if __name__ == "__main__":
    main()
