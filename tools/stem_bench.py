"""Stem forward and weight gradient: md2_stem_fwd / md2_stem_wgrad (stem_ops, forced on)
vs MIOpen's forward / backward-weights conv at the training step's shapes (B=12 C=3
depth encoder, B=24 C=6 pose encoder, 192x640).  Prints ms per call (HIP events); run
under rocprofv3 --kernel-trace for the per-kernel split.  python tools/stem_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monodepth2_amd import stem_ops  # noqa: E402


def run_fwd(B, C, use_ours, n=20):
    CL = torch.channels_last
    conv = torch.nn.Conv2d(C, 64, 7, 2, 3, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(B, C, 192, 640, device="cuda").contiguous(memory_format=CL)
    stem_ops.ENABLED = stem_ops.FWD_ENABLED = use_ours
    with torch.no_grad():
        for _ in range(3):
            stem_ops.stem_conv(conv, x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            stem_ops.stem_conv(conv, x)
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def run(B, C, use_ours, n=20):
    CL = torch.channels_last
    conv = torch.nn.Conv2d(C, 64, 7, 2, 3, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(B, C, 192, 640, device="cuda").contiguous(memory_format=CL)
    stem_ops.ENABLED = use_ours
    y = stem_ops.stem_conv(conv, x)
    g = torch.randn_like(y).contiguous(memory_format=CL)
    for _ in range(3):
        torch.autograd.grad(y, conv.weight, g, retain_graph=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        torch.autograd.grad(y, conv.weight, g, retain_graph=True)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for B, C in ((12, 3), (24, 6)):
    print(f"B={B} C={C}: wgrad ours {run(B, C, True):.3f} ms, MIOpen {run(B, C, False):.3f} ms; "
          f"fwd ours {run_fwd(B, C, True):.3f} ms, MIOpen {run_fwd(B, C, False):.3f} ms", flush=True)
