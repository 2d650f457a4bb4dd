import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from monodepth2_amd import conv_ops
CL = torch.channels_last
for (Co, Ci) in [(64, 64), (128, 128), (256, 256), (512, 512), (256, 512), (16, 16), (32, 96)]:
    x = torch.randn(2, Ci, 16, 16, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(Co, Ci, 3, 3, device="cuda").contiguous(memory_format=CL)
    for _ in range(3): conv_ops._split_weights(x, w, 1, 1, True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): conv_ops._split_weights(x, w, 1, 1, True)
    e1.record(); e1.synchronize()
    print(Co, Ci, round(e0.elapsed_time(e1) / 50 * 1e3, 1), "us", flush=True)
