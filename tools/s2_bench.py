"""Stride-2 input gradients: x6 parity classes (md2_conv_dgrad, stride 2) vs MIOpen at the
encoders' stride-2 shapes (depth B=12, pose B=24).  python tools/s2_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from conv_bench import CL, timeit  # noqa: E402
from monodepth2_amd import conv_ops  # noqa: E402

for B in (12, 24):
    for (C, N, k, p, H, W) in [(64, 128, 3, 1, 48, 160), (128, 256, 3, 1, 24, 80), (256, 512, 3, 1, 12, 40),
                               (64, 128, 1, 0, 48, 160), (128, 256, 1, 0, 24, 80), (256, 512, 1, 0, 12, 40)]:
        x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
        w = torch.randn(N, C, k, k, device="cuda").contiguous(memory_format=CL)
        gy = torch.randn(B, N, H // 2, W // 2, device="cuda").contiguous(memory_format=CL)
        gf = 2 * B * (H // 2) * (W // 2) * N * C * k * k / 1e9
        t6 = timeit(lambda: conv_ops._dgrad(gy, x, w, p, conv_ops.X6, 2))
        tm = timeit(lambda: conv_ops._miopen_bwd(gy, x, w, 2, p, (True, False, False))[0])
        print(f"B={B} {C}->{N} {k}x{k}/2 {H}x{W}: x6 {1e3 * t6:.1f} us ({gf / t6:.0f} TF)  "
              f"MIOpen {1e3 * tm:.1f} us ({gf / tm:.0f} TF)", flush=True)
