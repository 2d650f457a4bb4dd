"""Print the autograd node types between the loss and the pose network of one
training step (debug aid): python tools/autograd_graph.py"""
import sys

import torch

sys.path.insert(0, ".")


def main():
    from monodepth2_amd.data import synthetic_batch
    from monodepth2_amd.options import default_options
    from monodepth2_amd.trainer import Trainer
    opt = default_options(batch_size=2, height=64, width=128, num_layers=18, weights_init="scratch",
                          frame_ids=[0, -1, 1], log_dir="/tmp/md2_dbg", channels_last=True)
    tr = Trainer(opt, device=torch.device("cuda"), rank=0, world_size=1)
    batch = synthetic_batch(2, 64, 128, [0, -1, 1], 4, seed=1, device=torch.device("cuda"))
    tr.set_train()
    outputs, losses = tr.process_batch(batch)
    seen, order = set(), []
    stack = [(losses["loss"].grad_fn, 0)]
    while stack:
        fn, d = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        order.append((d, type(fn).__name__))
        for nxt, _ in fn.next_functions:
            stack.append((nxt, d + 1))
    counts = {}
    for d, n in order:
        counts[n] = counts.get(n, 0) + 1
    for n, c in sorted(counts.items(), key=lambda kv: -kv[1]):
        print(f"{c:5d} {n}")
    # the path from the loss down to the pose producer
    pose = [fn for fn in seen if "Pose" in type(fn).__name__]
    print("pose nodes:", [type(f).__name__ for f in pose])
    for fn in pose:
        q = [(fn, 0)]
        while q:
            f, d = q.pop()
            if f is None or d > 14:
                continue
            print("  " * d + type(f).__name__)
            for nxt, _ in f.next_functions:
                q.append((nxt, d + 1))


if __name__ == "__main__":
    main()
