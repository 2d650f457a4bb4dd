"""Per-shape autotune table of the training step's convolutions: for every (op,
shape) the timed candidates (x6 128 / x6 256 / f32 MFMA / MIOpen; the x6 candidates
only where the shape fits them), the one kept, its TFLOP/s, how often the step calls
it, and the step's time per op class on the kept candidates.

    python tools/conv_choices.py [--batch 12] [--steps 3] [out.json]
"""
import argparse
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import monodepth2_amd  # noqa: E402,F401
import torch  # noqa: E402

from monodepth2_amd import conv_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=12)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("out", nargs="?", default=None)
    args = ap.parse_args()
    sys.argv = [sys.argv[0], "--batch", str(args.batch), "--graph", "0"]
    import bench
    from monodepth2_amd.data import synthetic_batch
    bargs = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = bench.make_trainer(bargs, dev, 0, 1)
    batch = synthetic_batch(bargs.batch, bargs.height, bargs.width, tr.opt.frame_ids, 4, seed=100, device=dev,
                            eight_bit=True)
    tr.set_train()
    for _ in range(args.steps):
        tr.train_step(batch)
    torch.cuda.synchronize()
    # calls per step: count the forward keys of one more step
    calls = Counter()
    orig = conv_ops._Conv.forward

    def counting(ctx, x, weight, stride, pad):
        calls[(tuple(x.shape), tuple(weight.shape), stride, pad)] += 1
        return orig(ctx, x, weight, stride, pad)
    conv_ops._Conv.forward = staticmethod(counting)
    tr.train_step(batch)
    torch.cuda.synchronize()
    conv_ops._Conv.forward = staticmethod(orig)

    rows, per_op = [], Counter()
    for k, times in sorted(conv_ops._times.items(), key=lambda kv: kv[0]):
        op, xs, ws, s, p = k
        B, C, H, W = xs
        N, _, KH, KW = ws
        Ho, Wo = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
        fl = 2.0 * B * Ho * Wo * N * C * KH * KW
        names = list(times)
        kept = names[conv_ops._choice[k]]
        n = calls[(xs, ws, s, p)]
        row = {"op": op, "x": xs, "w": ws, "stride": s, "pad": p, "calls": n,
               "ms": {nm: round(t, 4) for nm, t in times.items()}, "kept": kept,
               "tflops_kept": round(fl / (times[kept] * 1e-3) / 1e12, 1)}
        rows.append(row)
        per_op[(op, kept == "miopen")] += n * times[kept]
        print(f"{op:5s} x{list(xs)} w{list(ws)} s{s} n{n} kept {kept:8s} {row['tflops_kept']:6.1f} TF  "
              + " ".join(f"{nm}={t:.3f}" for nm, t in times.items()))
    for (op, mi), t in sorted(per_op.items()):
        print(f"step total {op:5s} {'miopen' if mi else 'ours  '}: {t:.3f} ms")
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"rows": rows, "step_ms": {f"{op}/{'miopen' if mi else 'ours'}": round(t, 4)
                                                  for (op, mi), t in per_op.items()}}, f, indent=1)


if __name__ == "__main__":
    main()
