"""Disparity-head forward / backward at the step's four scales (B=12, 640x192),
HIP-event-timed averages over 50 calls.  python tools/head_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monodepth2_amd.decoder_ops import disp_head  # noqa: E402

CL = torch.channels_last
for C, h, w in [(16, 192, 640), (32, 96, 320), (64, 48, 160), (128, 24, 80)]:
    conv = torch.nn.Conv2d(C, 1, 3).cuda().to(memory_format=CL)
    P = torch.randn(12, C, h + 2, w + 2, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    g = torch.randn(12, 1, h, w, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            disp_head(P, conv)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        e0.record()
        for _ in range(50):
            disp_head(P, conv)
        e1.record()
    e1.synchronize()
    fwd = e0.elapsed_time(e1) / 50 * 1e3
    d = disp_head(P, conv)
    e0.record()
    for _ in range(20):
        torch.autograd.grad(d, (P, conv.weight, conv.bias), g, retain_graph=True)
    e1.record()
    e1.synchronize()
    bwd = e0.elapsed_time(e1) / 20 * 1e3
    gbs = P.numel() * 4 / (fwd * 1e-6) / 1e9
    print(f"C={C} {h}x{w}: fwd {fwd:.1f} us ({gbs:.0f} GB/s of input), bwd {bwd:.1f} us", flush=True)
