"""One weight-gradient shape, one kernel variant, repeated (for rocprofv3 counter passes).
    python tools/wgrad_one.py B Cin Cout pad H W flags [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, wgrad  # noqa: E402


def main():
    B, C, N, p, H, W, fl = (int(v) for v in sys.argv[1:8])
    reps = int(sys.argv[8]) if len(sys.argv) > 8 else 20
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(N, C, 3, 3, device="cuda").contiguous(memory_format=CL)
    gy = torch.randn_like(F.conv2d(x, w, None, 1, p)).contiguous(memory_format=CL)
    for _ in range(reps):
        wgrad(gy, x, w, 1, p, fl)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
