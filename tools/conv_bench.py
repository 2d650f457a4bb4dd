"""md2_conv_{fwd,dgrad,wgrad} (csrc/conv.hip, f32 MFMA implicit GEMM) vs MIOpen
(F.conv2d / aten.convolution_backward, channels_last fp32) on the training step's
convolution shapes: max relative error and time per call.
python tools/conv_bench.py [out.json]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import monodepth2_amd  # noqa: F401,E402  (MIOpen env)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from monodepth2_amd import _lib  # noqa: E402

CL = torch.channels_last

# (name, B, Cin, Cout, k, stride, pad, H, W)  — depth encoder at B=12; the pose
# encoder runs the same shapes at B=24; decoder convs see pre-padded inputs (pad 0)
SHAPES = [
    ("enc.layer1", 12, 64, 64, 3, 1, 1, 48, 160),
    ("enc.layer2", 12, 128, 128, 3, 1, 1, 24, 80),
    ("enc.layer3", 12, 256, 256, 3, 1, 1, 12, 40),
    ("enc.layer4", 12, 512, 512, 3, 1, 1, 6, 20),
    ("pose.layer1", 24, 64, 64, 3, 1, 1, 48, 160),
    ("pose.layer3", 24, 256, 256, 3, 1, 1, 12, 40),
    ("enc.layer2.0.conv1", 12, 64, 128, 3, 2, 1, 48, 160),
    ("enc.layer4.0.conv1", 12, 256, 512, 3, 2, 1, 12, 40),
    ("enc.layer2.0.down", 12, 64, 128, 1, 2, 0, 48, 160),
    ("dec.0", 12, 512, 256, 3, 1, 0, 8, 22),
    ("dec.1", 12, 512, 256, 3, 1, 0, 14, 42),
    ("dec.3", 12, 256, 128, 3, 1, 0, 26, 82),
    ("dec.5", 12, 128, 64, 3, 1, 0, 50, 162),
    ("dec.6", 12, 64, 32, 3, 1, 0, 50, 162),
    ("dec.7", 12, 96, 32, 3, 1, 0, 98, 322),
    ("dec.8", 12, 32, 16, 3, 1, 0, 98, 322),
    ("dec.9", 12, 16, 16, 3, 1, 0, 194, 642),
]

_WS = {}


def _ws(nb, dev):
    ws = _WS.get(nb)
    if ws is None:
        ws = _WS[nb] = torch.empty(max(nb, 4), dtype=torch.uint8, device=dev)
    return ws


def desc(x, w, stride, pad, flags=0):
    B, C, H, W = x.shape
    N, _, KH, KW = w.shape
    return _lib.ConvDesc(B, H, W, C, N, KH, KW, stride, pad, flags)


def fwd(x, w, stride, pad, flags=0):
    d = desc(x, w, stride, pad, flags)
    B, _, H, W = x.shape
    N, _, KH, KW = w.shape
    y = torch.empty(B, N, (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1, device=x.device,
                    memory_format=CL)
    ws = _ws(_lib.lib().md2_conv_workspace_bytes(ctypes.byref(d)), x.device)
    _lib.check(_lib.lib().md2_conv_fwd(ctypes.byref(d), x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream), "md2_conv_fwd")
    return y


def dgrad(gy, x, w, stride, pad, flags=0):
    d = desc(x, w, stride, pad, flags)
    gx = torch.empty_like(x, memory_format=CL)
    ws = _ws(_lib.lib().md2_conv_workspace_bytes(ctypes.byref(d)), x.device)
    _lib.check(_lib.lib().md2_conv_dgrad(ctypes.byref(d), gy.data_ptr(), w.data_ptr(), gx.data_ptr(), ws.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream), "md2_conv_dgrad")
    return gx


def wgrad(gy, x, w, stride, pad, flags=0):
    d = desc(x, w, stride, pad, flags)
    gw = torch.empty_like(w, memory_format=CL)
    ws = _ws(_lib.lib().md2_conv_workspace_bytes(ctypes.byref(d)), x.device)
    _lib.check(_lib.lib().md2_conv_wgrad(ctypes.byref(d), x.data_ptr(), gy.data_ptr(), gw.data_ptr(), ws.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream), "md2_conv_wgrad")
    return gw


def timeit(fn, n=20):
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


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


def main():
    torch.manual_seed(0)
    rows = []
    for name, B, C, N, k, s, p, H, W in SHAPES:
        x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
        w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
        y = F.conv2d(x, w, stride=s, padding=p)
        gy = torch.randn_like(y).contiguous(memory_format=CL)
        flops = 2.0 * y.numel() * C * k * k
        bw = lambda m: torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, m)  # noqa: E731
        gx_ref, gw_ref, _ = bw((True, True, False))
        r = {"name": name, "shape": [B, C, N, k, s, p, H, W], "gflop": round(flops / 1e9, 3)}
        r["fwd_err"] = rel(fwd(x, w, s, p), y)
        r["fwd_ms"] = timeit(lambda: fwd(x, w, s, p))
        r["fwd_miopen_ms"] = timeit(lambda: F.conv2d(x, w, stride=s, padding=p))
        if s == 1:
            r["dgrad_err"] = rel(dgrad(gy, x, w, s, p), gx_ref)
            r["dgrad_ms"] = timeit(lambda: dgrad(gy, x, w, s, p))
        r["dgrad_miopen_ms"] = timeit(lambda: bw((True, False, False)))
        r["wgrad_err"] = rel(wgrad(gy, x, w, s, p), gw_ref)
        r["wgrad_ms"] = timeit(lambda: wgrad(gy, x, w, s, p))
        r["wgrad_miopen_ms"] = timeit(lambda: bw((False, True, False)))
        for k2 in list(r):
            if k2.endswith("_ms"):
                r[k2] = round(r[k2], 4)
                r[k2.replace("_ms", "_tf")] = round(flops / r[k2] / 1e9, 1)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
