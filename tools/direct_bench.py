"""The DepthDecoder's 16-output-channel 3x3 convolutions (upconv(0,1) 16->16 at 192x640
and upconv(0,0) 32->16 at 96x320 on their reflection-padded inputs, batch 12) and their
input gradients: md2_conv_direct's f32 VALU form vs its split-bf16 MFMA form (X6) vs
MIOpen.  Prints ms per call (HIP events).  python tools/direct_bench.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monodepth2_amd import conv_ops  # noqa: E402

CL = torch.channels_last


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for C, N, H, W in ((16, 16, 194, 642), (32, 16, 98, 322)):
    x = torch.randn(12, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / (9 * C) ** 0.5).contiguous(memory_format=CL)
    gy = torch.randn(12, N, H - 2, W - 2, device="cuda").contiguous(memory_format=CL)
    f = {"valu": timed(lambda: conv_ops._direct_fwd(x, w, 0)),
         "x6": timed(lambda: conv_ops._direct_fwd(x, w, 0, conv_ops.X6)),
         "miopen": timed(lambda: F.conv2d(x, w))}
    d = {"valu": timed(lambda: conv_ops._direct_dgrad(gy, w, 0)),
         "x6": timed(lambda: conv_ops._direct_dgrad(gy, w, 0, conv_ops.X6)),
         "miopen": timed(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (0, 0), (1, 1), False,
                                                                     (0, 0), 1, (True, False, False)))}
    wg = {"valu": timed(lambda: conv_ops._direct_wgrad(gy, x, w, 0)),
          "x6": timed(lambda: conv_ops._direct_wgrad(gy, x, w, 0, conv_ops.X6)),
          "x6pw": timed(lambda: conv_ops._wgrad(gy, x, w, 1, 0, conv_ops.X6 | conv_ops.PATCH)),
          "miopen": timed(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (0, 0), (1, 1), False,
                                                                      (0, 0), 1, (False, True, False)))}
    print(f"{C}->{N} {H}x{W}: fwd " + ", ".join(f"{k} {v:.4f}" for k, v in f.items()) +
          " ms; dgrad " + ", ".join(f"{k} {v:.4f}" for k, v in d.items()) +
          " ms; wgrad " + ", ".join(f"{k} {v:.4f}" for k, v in wg.items()) + " ms", flush=True)
