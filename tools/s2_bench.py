"""Stride-2 input gradients of the step: per-class x6 launches vs the one-launch form
(MD2_CONV_S2_ONE) vs one GEMM + gather (conv_ops._dgrad_col) vs MIOpen, ms per call.
    python tools/s2_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, dgrad, timeit, rel  # noqa: E402
from monodepth2_amd import _lib, conv_ops  # noqa: E402

X6, ONE, B256 = _lib.CONV_X6, _lib.CONV_S2_ONE, _lib.CONV_BM256
SHAPES = [(12, 64, 128, 3, 1, 48, 160), (12, 128, 256, 3, 1, 24, 80), (12, 256, 512, 3, 1, 12, 40),
          (24, 64, 128, 3, 1, 48, 160), (24, 128, 256, 3, 1, 24, 80), (12, 64, 128, 1, 0, 48, 160)]


def main():
    torch.manual_seed(0)
    for B, C, N, k, p, H, W in SHAPES:
        x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
        w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
        gy = torch.randn_like(F.conv2d(x, w, None, 2, p)).contiguous(memory_format=CL)
        mi = lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (2, 2), (p, p), (1, 1), False, (0, 0), 1,
                                                         (True, False, False))[0]
        ref = mi()
        row = {"shape": [B, C, N, k, p, H, W]}
        for tag, fl in (("x6_s2", X6), ("one", X6 | ONE), ("one_256", X6 | ONE | B256)):
            row[tag] = round(timeit(lambda: dgrad(gy, x, w, 2, p, fl)), 4)
            row["err_" + tag] = float(rel(dgrad(gy, x, w, 2, p, fl), ref))
        for tag, fl in (("col", X6), ("col_256", X6 | B256)):
            row[tag] = round(timeit(lambda: conv_ops._dgrad_col(gy, x, w, 2, p, fl)), 4)
            row["err_" + tag] = float(rel(conv_ops._dgrad_col(gy, x, w, 2, p, fl), ref))
        row["miopen"] = round(timeit(mi), 4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
