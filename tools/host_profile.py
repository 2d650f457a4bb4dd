"""Where the host time of one training step goes: torch.profiler (CPU activities)
over a few steps of the bench configuration, self CPU time per op, top N.

    python tools/host_profile.py [--steps 5] [--top 40]
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
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--channels-last", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    opt = default_options(batch_size=12, height=192, width=640, weights_init="scratch", log_dir="/tmp/md2_hp",
                          channels_last=a.channels_last)
    tr = Trainer(opt, device=dev)
    batch = synthetic_batch(12, 192, 640, opt.frame_ids, 4, seed=1, device=dev)
    tr.set_train()
    for _ in range(8):
        tr.train_step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(a.steps):
            tr.train_step(batch)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    total = sum(e.self_cpu_time_total for e in ka)
    print(f"host self time per step: {total / a.steps / 1e3:.2f} ms over {sum(e.count for e in ka) // a.steps} events")
    rows = sorted(ka, key=lambda e: -e.self_cpu_time_total)[:a.top]
    for e in rows:
        print(f"{e.key[:70]:70s} {e.count // a.steps:6d}/step {e.self_cpu_time_total / a.steps / 1e3:8.3f} ms/step "
              f"{e.self_cpu_time_total / max(e.count, 1):8.1f} us/call")


if __name__ == "__main__":
    main()
