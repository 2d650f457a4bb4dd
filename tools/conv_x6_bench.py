"""Split-bf16 (x6) vs exact-f32 MFMA vs MIOpen on the step's convolution shapes:
time per call and error against an fp64 reference (max |err| / max |ref| and
relative L2).  python tools/conv_x6_bench.py [modes]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json  # noqa: E402

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import CL, SHAPES, fwd, dgrad, wgrad, timeit  # noqa: E402
from monodepth2_amd import _lib  # noqa: E402

X6 = _lib.CONV_X6


def errs(a, ref):
    d = (a.double() - ref)
    return float(d.abs().max() / ref.abs().max()), float(d.norm() / ref.norm())


def main():
    torch.manual_seed(0)
    modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fwd"]
    for name, B, C, N, k, s, p, H, W in SHAPES:
        x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
        w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
        gf = 2 * B * ((H + 2 * p - k) // s + 1) * ((W + 2 * p - k) // s + 1) * N * C * k * k / 1e9
        row = {"name": name, "gflop": round(gf, 3)}
        if "quickw" in modes:   # x6 weight-gradient timings only
            gy = torch.randn_like(F.conv2d(x, w, None, s, p)).contiguous(memory_format=CL)
            row["wgrad_x6_tf"] = round(gf / timeit(lambda: wgrad(gy, x, w, s, p, X6)), 1)
            print(json.dumps(row), flush=True)
            continue
        if "s3" in modes:   # x6 forward / patch forward / per-tap weight gradient (layout A/B)
            gy = torch.randn_like(F.conv2d(x, w, None, s, p)).contiguous(memory_format=CL)
            row["fwd_x6_tf"] = round(gf / timeit(lambda: fwd(x, w, s, p, X6)), 1)
            if k == 3 and s == 1:
                row["fwd_x6p_tf"] = round(gf / timeit(lambda: fwd(x, w, s, p, X6 | _lib.CONV_PATCH)), 1)
            row["wgrad_x6_tf"] = round(gf / timeit(lambda: wgrad(gy, x, w, s, p, X6)), 1)
            print(json.dumps(row), flush=True)
            continue
        if "quick" in modes:   # x6 timings only (A/B of variant builds)
            row["fwd_x6_tf"] = round(gf / timeit(lambda: fwd(x, w, s, p, X6)), 1)
            row["fwd_x6_256_tf"] = round(gf / timeit(lambda: fwd(x, w, s, p, X6 | _lib.CONV_BM256)), 1)
            if s == 1:
                gy = torch.randn_like(F.conv2d(x, w, None, s, p)).contiguous(memory_format=CL)
                row["dgrad_x6_tf"] = round(gf / timeit(lambda: dgrad(gy, x, w, s, p, X6)), 1)
            print(json.dumps(row), flush=True)
            continue
        if "fwd" in modes:
            ref = F.conv2d(x.double().cpu(), w.double().cpu(), None, s, p).cuda() if gf < 8 else \
                F.conv2d(x.double(), w.double(), None, s, p)
            t_x6 = timeit(lambda: fwd(x, w, s, p, X6))
            t_256 = timeit(lambda: fwd(x, w, s, p, X6 | _lib.CONV_BM256))
            row["fwd_x6_256_tf"] = round(gf / t_256, 1)
            row["err_x6_256"] = errs(fwd(x, w, s, p, X6 | _lib.CONV_BM256), ref)
            t_f32 = timeit(lambda: fwd(x, w, s, p))
            t_mi = timeit(lambda: F.conv2d(x, w, None, s, p))
            row.update({"fwd_x6_tf": round(gf / t_x6, 1), "fwd_f32_tf": round(gf / t_f32, 1),
                        "fwd_miopen_tf": round(gf / t_mi, 1),
                        "err_x6": errs(fwd(x, w, s, p, X6), ref), "err_f32": errs(fwd(x, w, s, p), ref),
                        "err_miopen": errs(F.conv2d(x, w, None, s, p), ref)})
        if "dgrad" in modes and s == 1:
            y = F.conv2d(x, w, None, s, p)
            gy = torch.randn_like(y).contiguous(memory_format=CL)
            gyd, xd, wd = gy.double(), x.double(), w.double()
            ref = torch.ops.aten.convolution_backward(gyd.cpu(), xd.cpu(), wd.cpu(), None, (s, s), (p, p), (1, 1), False,
                                                      (0, 0), 1, (True, False, False))[0].cuda()
            mi = lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False,  # noqa: E731
                                                             (0, 0), 1, (True, False, False))[0]
            t_x6 = timeit(lambda: dgrad(gy, x, w, s, p, X6))
            row["dgrad_x6_256_tf"] = round(gf / timeit(lambda: dgrad(gy, x, w, s, p, X6 | _lib.CONV_BM256)), 1)
            t_f32 = timeit(lambda: dgrad(gy, x, w, s, p))
            t_mi = timeit(mi)
            row.update({"dgrad_x6_tf": round(gf / t_x6, 1), "dgrad_f32_tf": round(gf / t_f32, 1),
                        "dgrad_miopen_tf": round(gf / t_mi, 1),
                        "dgrad_err_x6": errs(dgrad(gy, x, w, s, p, X6), ref),
                        "dgrad_err_f32": errs(dgrad(gy, x, w, s, p), ref), "dgrad_err_miopen": errs(mi(), ref)})
        if "wgrad" in modes:
            y = F.conv2d(x, w, None, s, p)
            gy = torch.randn_like(y).contiguous(memory_format=CL)
            ref = torch.ops.aten.convolution_backward(gy.double().cpu(), x.double().cpu(), w.double().cpu(), None, (s, s),
                                                      (p, p), (1, 1), False, (0, 0), 1, (False, True, False))[1].cuda()
            mi = lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False,  # noqa: E731
                                                             (0, 0), 1, (False, True, False))[1]
            t_x6 = timeit(lambda: wgrad(gy, x, w, s, p, X6))
            t_f32 = timeit(lambda: wgrad(gy, x, w, s, p))
            t_mi = timeit(mi)
            row.update({"wgrad_x6_tf": round(gf / t_x6, 1), "wgrad_f32_tf": round(gf / t_f32, 1),
                        "wgrad_miopen_tf": round(gf / t_mi, 1),
                        "wgrad_err_x6": errs(wgrad(gy, x, w, s, p, X6), ref),
                        "wgrad_err_miopen": errs(mi(), ref)})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
