"""md2_conv_direct vs x6 / MIOpen on the DepthDecoder's 16-output-channel layers
(forward and input gradient, B=12 640x192).  python tools/direct_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, timeit  # noqa: E402
from monodepth2_amd import conv_ops  # noqa: E402

for name, C, N, H, W in [("dec.8 32->16", 32, 16, 98, 322), ("dec.9 16->16", 16, 16, 194, 642)]:
    x = torch.randn(12, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / (9 * C) ** 0.5).contiguous(memory_format=CL)
    gy = torch.randn(12, N, H - 2, W - 2, device="cuda").contiguous(memory_format=CL)
    gf = 2 * 12 * (H - 2) * (W - 2) * N * C * 9 / 1e9
    wk = w.permute(2, 3, 1, 0).contiguous()
    wkd = w.flip(2, 3).permute(2, 3, 0, 1).contiguous()
    r = {"fwd direct": timeit(lambda: conv_ops._direct(x, wk, 0, N)),
         "fwd miopen": timeit(lambda: F.conv2d(x, w)),
         "fwd x6": timeit(lambda: conv_ops._fwd(x, w, 1, 0, conv_ops.X6)),
         "dgrad direct": timeit(lambda: conv_ops._direct(gy, wkd, 2, C)),
         "dgrad miopen": timeit(lambda: conv_ops._miopen_bwd(gy, x, w, 1, 0, (True, False, False))[0]),
         "dgrad x6": timeit(lambda: conv_ops._dgrad(gy, x, w, 0, conv_ops.X6)),
         "wgrad direct": timeit(lambda: conv_ops._direct_wgrad(gy, x, w, 0)),
         "wgrad miopen": timeit(lambda: conv_ops._miopen_bwd(gy, x, w, 1, 0, (False, True, False))[1]),
         "wgrad x6": timeit(lambda: conv_ops._wgrad(gy, x, w, 1, 0, conv_ops.X6))}
    print(name, "  ".join(f"{k} {1e3 * v:.1f} us ({gf / v:.0f} TF)" for k, v in r.items()), flush=True)
