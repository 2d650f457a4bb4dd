"""conv1 (7x7 stride 2 pad 3 -> 64) forward + weight gradient (the input is data: no
input gradient) under MIOpen for layouts and channel paddings: C=3 (depth) / 6 (pose)
as is, zero-padded to 4 / 8, NCHW vs channels_last.  python tools/conv1_variants.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import monodepth2_amd  # noqa: E402,F401


def bench(B, C, Cpad, cl, H=192, W=640, n=10):
    dev = torch.device("cuda")
    fmt = torch.channels_last if cl else torch.contiguous_format
    w = torch.randn(64, C, 7, 7, device=dev).contiguous(memory_format=fmt).requires_grad_(True)
    x = torch.randn(B, Cpad, H, W, device=dev).contiguous(memory_format=fmt)

    def step():
        wp = F.pad(w, (0, 0, 0, 0, 0, Cpad - C)) if Cpad != C else w
        if cl:
            wp = wp.contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, wp, None, 2, 3)
        g, = torch.autograd.grad(y, w, torch.ones_like(y))
        return y, g
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        step()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for B, C in ((12, 3), (24, 6)):
    for Cpad in (C, C + 1 if C == 3 else 8):
        for cl in (True, False):
            t = bench(B, C, Cpad, cl)
            print(f"B={B} C={C} pad->{Cpad} {'NHWC' if cl else 'NCHW'}: fwd+wgrad {t:.3f} ms", flush=True)
