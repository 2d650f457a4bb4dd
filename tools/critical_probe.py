"""Which stream's chain sets the two-stream step?  A latency probe: a one-wave spin
kernel (torch.cuda._sleep, no throughput taken from the other stream) inserted into one
chain's backward — at the start of the depth network's backward (the main stream,
right after the hot path's backward) or of the pose network's (its stream) — and the
eager step time with and without it.  If adding D ms to a chain adds D ms to the step,
that chain is the critical path; if the step does not move, the chain has that much
slack.

    python tools/critical_probe.py [--ms 0.5] [--steps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


class _Spin(torch.autograd.Function):
    cycles = 0

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if _Spin.cycles:
            torch.cuda._sleep(_Spin.cycles)
        return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--graph", "0"]
    import bench
    from monodepth2_amd.data import synthetic_batch
    args = bench.parse()
    dev = torch.device("cuda", 0)
    tr = bench.make_trainer(args, dev, 0, 1)
    batch = synthetic_batch(args.batch, args.height, args.width, tr.opt.frame_ids, 4, seed=100, device=dev,
                            eight_bit=True)
    where = {"depth": False, "pose": False}
    depth, pose = tr.models["depth"], tr.models["pose"]
    dfwd, pfwd = depth.forward, pose.forward

    def depth_forward(*x, **k):
        out = dfwd(*x, **k)
        if where["depth"]:   # the disparities' gradient arrives first in the depth backward
            out = {key: (_Spin.apply(v) if key == ("disp", 0) else v) for key, v in out.items()}
        return out

    def pose_forward(*x, **k):
        out = pfwd(*x, **k)
        if where["pose"]:
            # one spin on the pose output's gradient (a packed tensor, or the axis-angle)
            out = _Spin.apply(out) if torch.is_tensor(out) else (_Spin.apply(out[0]),) + tuple(out[1:])
        return out
    depth.forward, pose.forward = depth_forward, pose_forward

    # spin cycles per ms, measured
    _Spin.cycles = 1_000_000
    for _ in range(2):
        torch.cuda._sleep(_Spin.cycles)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(_Spin.cycles)
    e1.record()
    e1.synchronize()
    per_ms = _Spin.cycles / e0.elapsed_time(e1)
    _Spin.cycles = int(per_ms * a.ms)

    def timed():
        for _ in range(5):
            tr.train_step(batch)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.steps):
            tr.train_step(batch)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / a.steps

    for _ in range(5):
        tr.train_step(batch)
    for rep in range(2):
        for mode in ("none", "depth", "pose", "both"):
            where["depth"] = mode in ("depth", "both")
            where["pose"] = mode in ("pose", "both")
            print("rep %d, +%.2f ms spin in the %-5s backward: step %.3f ms" % (rep, a.ms, mode, timed()), flush=True)


if __name__ == "__main__":
    main()
