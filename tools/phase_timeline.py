"""Where the two streams' time goes in an eager training step (bench configuration):
HIP events, recorded without a profiler (rocprofv3 serialises the two streams), at

    start (main) | depth forward done (main) | pose forward done (pose stream)
    | losses done (main) | backward enqueued: pose stream done, main done | Adam done

averaged over the timed steps, as milliseconds from the step's start.  The backward
phase's two chains (depth network on the main stream, pose network on its own) end at
"bwd pose" / "bwd main"; the longer one is the step's critical path there.

    python tools/phase_timeline.py [--steps 20] [--batch 12]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=12)
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--batch", str(a.batch), "--graph", "0"]
    import bench
    from monodepth2_amd.data import synthetic_batch
    args = bench.parse()
    dev = torch.device("cuda", 0)
    tr = bench.make_trainer(args, dev, 0, 1)
    batch = synthetic_batch(args.batch, args.height, args.width, tr.opt.frame_ids, 4, seed=100, device=dev,
                            eight_bit=True)
    marks = {}

    def mark(name, stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream or torch.cuda.current_stream(dev))
        marks.setdefault(name, []).append(e)

    depth = tr.models["depth"]
    dfwd = depth.forward

    def depth_forward(*x, **k):
        out = dfwd(*x, **k)
        mark("depth fwd")
        return out
    depth.forward = depth_forward
    pp = tr.predict_poses

    def predict_poses(*x, **k):
        out = pp(*x, **k)
        mark("pose fwd")   # the pose stream (predict_poses runs inside its stream context)
        return out
    tr.predict_poses = predict_poses
    pb = tr.process_batch

    def process_batch(*x, **k):
        out = pb(*x, **k)
        mark("losses")
        return out
    tr.process_batch = process_batch
    loss_backward = torch.Tensor.backward

    def backward(self, *x, **k):
        r = loss_backward(self, *x, **k)
        if tr._pose_stream is not None:
            mark("bwd pose stream", tr._pose_stream)
        mark("bwd main")
        return r
    torch.Tensor.backward = backward

    for _ in range(8):
        tr.train_step(batch)
    torch.cuda.synchronize()
    marks.clear()
    starts, ends = [], []
    for _ in range(a.steps):
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        starts.append(s)
        tr.train_step(batch)
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ends.append(e)
    torch.cuda.synchronize()
    n = len(starts)
    print("step %.3f ms" % (sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / n))
    for name, evs in marks.items():
        k = len(evs) // n   # events per step
        for j in range(k):
            t = sum(starts[i].elapsed_time(evs[i * k + j]) for i in range(n)) / n
            print("  %-18s %7.3f ms" % (name + ("" if k == 1 else " #%d" % j), t))


if __name__ == "__main__":
    main()
