"""Disparity-head forward / backward at the step's four scales (B=12, 640x192),
HIP-event-timed averages over 50 back-to-back calls of md2_disp_head_fwd /
md2_disp_head_bwd through the C ABI (no autograd: its host overhead per call is
larger than the backward kernels themselves).  python tools/head_bench.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monodepth2_amd import _lib  # noqa: E402

CL = torch.channels_last
L = _lib.lib()
st = _lib.stream(torch.device("cuda", 0))
for C, h, w in [(16, 192, 640), (32, 96, 320), (64, 48, 160), (128, 24, 80)]:
    B = 12
    P = torch.randn(B, C, h + 2, w + 2, device="cuda").contiguous(memory_format=CL)
    weight = torch.randn(1, C, 3, 3, device="cuda").contiguous(memory_format=CL) * 0.05
    bias = torch.zeros(1, device="cuda")
    d = _lib.HeadDesc(B, C, h, w, _lib.HEAD_WEIGHT_CL)
    disp = torch.empty(B, 1, h, w, device="cuda")
    g = torch.randn(B, 1, h, w, device="cuda")
    gP = torch.empty_like(P, memory_format=CL)
    gw = torch.empty_like(weight)
    gb = torch.empty(1, device="cuda")
    ws = torch.empty(L.md2_disp_head_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device="cuda")

    def fwd():
        _lib.check(L.md2_disp_head_fwd(ctypes.byref(d), P.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                                       disp.data_ptr(), st), "md2_disp_head_fwd")

    def bwd():
        _lib.check(L.md2_disp_head_bwd(ctypes.byref(d), P.data_ptr(), weight.data_ptr(), disp.data_ptr(),
                                       g.data_ptr(), gP.data_ptr(), gw.data_ptr(), gb.data_ptr(), ws.data_ptr(), st),
                   "md2_disp_head_bwd")

    res = []
    for fn in (fwd, bwd):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / 50 * 1e3)
    print(f"C={C} {h}x{w}: fwd {res[0]:.1f} us, bwd {res[1]:.1f} us "
          f"(gP sum {float(gP.double().sum()):.6e}, gw sum {float(gw.double().sum()):.6e})", flush=True)
