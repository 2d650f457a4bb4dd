"""Device time per convolution shape in one training step (bench configuration).

torch.profiler with device activities over a few steps; convolution forward /
backward ops grouped by input shape, with each group's device time per step and
its fp32 MFMA rate (2·M·N·K per direction) so the inefficient layers stand out.

    python tools/conv_profile.py [--steps 5] [--stream-serial 1]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import monodepth2_amd  # noqa: F401,E402
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--batch", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    opt = default_options(batch_size=a.batch, height=192, width=640, weights_init="scratch",
                          log_dir="/tmp/md2_cp")
    tr = Trainer(opt, device=dev)
    batch = synthetic_batch(a.batch, 192, 640, opt.frame_ids, 4, seed=1, device=dev)
    tr.set_train()
    for _ in range(6):
        tr.train_step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(a.steps):
            tr.train_step(batch)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    rows = []
    for e in ka:
        if e.key not in ("aten::convolution", "aten::convolution_backward"):
            continue
        dt = getattr(e, "device_time_total", None)
        if dt is None:
            dt = e.cuda_time_total
        rows.append((dt / a.steps / 1e3, e.count / a.steps, e.key, e.input_shapes))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"conv device time per step: {tot:.3f} ms")
    for ms, cnt, key, shp in rows[:a.top]:
        x, w = shp[0], shp[1]
        if key == "aten::convolution_backward":
            x, w = shp[1], shp[2]
        try:
            n, c, h, wd = x
            co, ci, kh, kw = w
            # output size from stride guess: read from the forward shapes list when present
            print(f"{ms:7.3f} ms {cnt:4.1f}/step {key[6:]:22s} x={x} w={w}")
        except Exception:
            print(f"{ms:7.3f} ms {cnt:4.1f}/step {key[6:]:22s} {shp}")


if __name__ == "__main__":
    main()
