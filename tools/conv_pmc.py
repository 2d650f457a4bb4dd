"""Run one convolution shape through md2_conv_fwd/dgrad/wgrad and MIOpen repeatedly
(for rocprofv3 --pmc passes).  python tools/conv_pmc.py B C N k s p H W [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, fwd, dgrad, wgrad  # noqa: E402
from monodepth2_amd import _lib  # noqa: E402

FL = _lib.CONV_X6 if os.environ.get("X6") else 0
ONLY_FWD = bool(os.environ.get("ONLY_FWD"))

B, C, N, k, s, p, H, W = (int(v) for v in sys.argv[1:9])
iters = int(sys.argv[9]) if len(sys.argv) > 9 else 20
x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
w = torch.randn(N, C, k, k, device="cuda").contiguous(memory_format=CL)
y = F.conv2d(x, w, None, s, p)
gy = torch.randn_like(y).contiguous(memory_format=CL)
for _ in range(iters):
    fwd(x, w, s, p, FL)
    F.conv2d(x, w, None, s, p)
    if ONLY_FWD:
        continue
    if s == 1:
        dgrad(gy, x, w, p)
    wgrad(gy, x, w, s, p)
    torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (True, True, False))
torch.cuda.synchronize()
