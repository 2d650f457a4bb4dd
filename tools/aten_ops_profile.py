"""Which ATen ops (not our HIP kernels) run inside an eager training step, with their
input shapes and device time: torch.profiler over a few steps of the default bench
trainer.  python tools/aten_ops_profile.py"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0], "--graph", "0"]
import bench  # noqa: E402
from monodepth2_amd.data import synthetic_batch  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
tr = bench.make_trainer(args, dev, 0, 1)
batch = synthetic_batch(args.batch, args.height, args.width, tr.opt.frame_ids, 4, seed=100, device=dev, eight_bit=True)
tr.set_train()
for _ in range(4):
    tr.train_step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for _ in range(2):
        tr.train_step(batch)
    torch.cuda.synchronize()
keep = ("aten::add", "aten::copy_", "aten::cat", "aten::fill_", "aten::zero_", "aten::mul", "aten::contiguous",
        "aten::clone", "aten::flip", "aten::mean", "aten::sum", "aten::to", "aten::_to_copy", "aten::index")
rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith(keep)]
rows.sort(key=lambda e: -e.device_time_total)
for e in rows[:40]:
    print(f"{e.device_time_total / 2:9.1f} us/step  n={e.count // 2:3d}  {e.key:28s} {str(e.input_shapes)[:150]}", flush=True)
