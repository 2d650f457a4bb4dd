"""Which stream each parameter's gradient is accumulated on, per training step, eager and
captured, and whether autograd warns of an AccumulateGrad stream mismatch (the capture
must run on the warm-up stream: trainer._capture).  python tools/accgrad_streams.py"""
import os, sys, warnings
sys.path.insert(0, os.getcwd())
import torch
from monodepth2_amd.options import default_options
from monodepth2_amd.trainer import Trainer
from monodepth2_amd.data import synthetic_batch

def run(graph, pose_streams=1):
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=2, height=64, width=128, weights_init="scratch", log_dir="/tmp/md2d",
                                 frame_ids=[0, -1, 1], hip_graph=graph, pose_streams=pose_streams),
                 device=torch.device("cuda", 0))
    batch = synthetic_batch(2, 64, 128, tr.opt.frame_ids, 4, seed=3, device="cuda")
    tr.set_train()
    main = torch.cuda.current_stream()
    pose_names = {id(p): n for n, p in tr.nets.named_parameters() if "pose" in n}
    seen = {}
    def hook(p):
        s = torch.cuda.current_stream()
        seen.setdefault((id(p) in pose_names, s.cuda_stream), 0)
        seen[(id(p) in pose_names, s.cuda_stream)] += 1
    hs = [p.register_post_accumulate_grad_hook(hook) for p in tr.nets.parameters() if p.requires_grad]
    for i in range(4):
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            seen.clear()
            tr.train_step(batch)
            torch.cuda.synchronize()
        msgs = [str(x.message)[:60] for x in w if "AccumulateGrad" in str(x.message)]
        print(f"graph={graph} pose_streams={pose_streams} step {i}: mismatch warnings={len(msgs)} "
              f"acc streams (pose?, stream)->count {seen} main={main.cuda_stream} "
              f"pose={tr._pose_stream.cuda_stream if tr._pose_stream is not None else None}", flush=True)
    for h in hs: h.remove()

run(False)
run(True)
run(False, 0)
