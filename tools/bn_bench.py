"""BatchNorm(+residual)+ReLU forward and backward (bn_ops.bn_act -> md2_bn_*) at the
depth encoder's shapes (batch 12, 192x640: stem 64@96x320, layers 64@48x160 ..
512@6x20), ms per layer pass (fwd + bwd, HIP events); run under rocprofv3
--kernel-trace --stats for the per-kernel split.  python tools/bn_bench.py"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monodepth2_amd import bn_ops  # noqa: E402

CL = torch.channels_last
SHAPES = [(64, 96, 320), (64, 48, 160), (128, 24, 80), (256, 12, 40), (512, 6, 20)]


def main(n=20):
    torch.manual_seed(0)
    tot = 0.0
    for C, H, W in SHAPES:
        bn = nn.BatchNorm2d(C).cuda().train()
        x = torch.randn(12, C, H, W, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
        r = torch.randn_like(x)
        g = torch.randn_like(x)

        def step():
            y = bn_ops.bn_act(bn, x, r)
            torch.autograd.grad(y, (x, bn.weight), g)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        tot += ms
        print(f"C={C} {H}x{W}: {ms:.4f} ms", flush=True)
    print(f"total {tot:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
