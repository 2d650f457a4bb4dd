"""Per-tap x6 kernel vs the patch-staged x6 kernel (MD2_CONV_PATCH) vs MIOpen on the
step's 3x3 stride-1 shapes: forward and input gradient, TFLOP/s (f32-equivalent).
    python tools/patch_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, SHAPES, fwd, dgrad, timeit  # noqa: E402
from monodepth2_amd import _lib  # noqa: E402

X6, B256, P = _lib.CONV_X6, _lib.CONV_BM256, _lib.CONV_PATCH
EXTRA = [("pose.layer1", 24, 64, 64, 3, 1, 1, 48, 160), ("pose.layer2", 24, 128, 128, 3, 1, 1, 24, 80),
         ("pose.layer4", 24, 512, 512, 3, 1, 1, 6, 20)]


def main():
    torch.manual_seed(0)
    for name, B, C, N, k, s, p, H, W in list(SHAPES) + EXTRA:
        if k != 3 or s != 1 or C % 32:
            continue
        x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
        w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
        gf = 2 * B * (H + 2 * p - 2) * (W + 2 * p - 2) * N * C * 9 / 1e9
        row = {"name": name, "shape": [B, C, N, p, H, W], "gflop": round(gf, 2)}
        for tag, fl in (("x6", X6), ("x6_256", X6 | B256), ("x6p", X6 | P), ("x6p_256", X6 | P | B256)):
            row["fwd_" + tag] = round(gf / timeit(lambda: fwd(x, w, s, p, fl)), 1)
        row["fwd_miopen"] = round(gf / timeit(lambda: F.conv2d(x, w, None, s, p)), 1)
        if N % 32 == 0:
            gy = torch.randn_like(F.conv2d(x, w, None, s, p)).contiguous(memory_format=CL)
            for tag, fl in (("x6", X6), ("x6_256", X6 | B256), ("x6p", X6 | P), ("x6p_256", X6 | P | B256)):
                row["dgrad_" + tag] = round(gf / timeit(lambda: dgrad(gy, x, w, s, p, fl)), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
