"""Run one md2_conv_fwd shape repeatedly (for rocprofv3 PMC passes).
python tools/conv_prof.py B C N k s p H W [narrow] [nosplit] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from conv_bench import CL, fwd as ours  # noqa: E402

B, C, N, k, s, p, H, W = (int(v) for v in sys.argv[1:9])
narrow = len(sys.argv) > 9 and sys.argv[9] == "1"
nosplit = len(sys.argv) > 10 and sys.argv[10] == "1"
iters = int(sys.argv[11]) if len(sys.argv) > 11 else 20
x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
w = torch.randn(N, C, k, k, device="cuda").contiguous(memory_format=CL)
for _ in range(iters):
    ours(x, w, s, p, narrow=narrow, nosplit=nosplit)
torch.cuda.synchronize()
