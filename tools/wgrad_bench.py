"""Weight gradients of the step's 3x3 stride-1 convolutions: the per-tap x6 kernel vs
the patch-staged one (MD2_CONV_PATCH, conv_x6pw_kernel) vs the warp-specialised one
(MD2_CONV_WS, conv_x6wws_kernel; every shape with more than 64 output channels, strided
too) vs MIOpen, TFLOP/s
(f32-equivalent), with each x6 result's relative error against MIOpen.
    python tools/wgrad_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, SHAPES, timeit, wgrad, rel  # noqa: E402
from monodepth2_amd import _lib  # noqa: E402

X6, P, WS, B256 = _lib.CONV_X6, _lib.CONV_PATCH, _lib.CONV_WS, _lib.CONV_BM256
EXTRA = [("pose.layer2", 24, 128, 128, 3, 1, 1, 24, 80), ("pose.layer4", 24, 512, 512, 3, 1, 1, 6, 20)]


def main():
    torch.manual_seed(0)
    for name, B, C, N, k, s, p, H, W in list(SHAPES) + EXTRA:
        if C % 8 or N % 8:
            continue
        x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
        w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
        gy = torch.randn_like(F.conv2d(x, w, None, s, p)).contiguous(memory_format=CL)
        gf = 2 * gy.shape[0] * gy.shape[2] * gy.shape[3] * N * C * k * k / 1e9
        row = {"name": name, "shape": [B, C, N, p, H, W], "gflop": round(gf, 2)}
        mi = lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                                         (False, True, False))[1]
        ref = mi()
        tags = [("x6", X6)] + ([("x6ws", X6 | WS), ("x6ws_256", X6 | WS | B256)] if N > 64 else []) + ([("x6pw", X6 | P)] if k == 3 and s == 1 else [])
        for tag, fl in tags:
            row[tag] = round(gf / timeit(lambda: wgrad(gy, x, w, s, p, fl)), 1)
            row["err_" + tag] = float(rel(wgrad(gy, x, w, s, p, fl), ref))
        row["miopen"] = round(gf / timeit(mi), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
