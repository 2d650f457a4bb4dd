"""Is MIOpen's bf16 input gradient of the pose decoder's last 1x1 convolution (256 -> 12,
B=64 pairs at 6x20: C5's pose_2) bitwise repeatable?  Runs it N times on one input and
counts the runs whose bits differ from the first; the same for the GEMM form
(conv_ops._dgrad_mm_bf16).  python tools/miopen_det_check.py [--runs 200]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=200)
    a = ap.parse_args()
    from monodepth2_amd import conv_ops
    torch.manual_seed(0)
    cl = torch.channels_last
    for (B, C, N, H, W, k, p) in [(64, 256, 12, 6, 20, 1, 0), (64, 256, 256, 6, 20, 3, 1), (32, 512, 512, 6, 20, 3, 1)]:
        x = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(N, C, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
        gy = torch.randn(B, N, H + 2 * p - k + 1, W + 2 * p - k + 1, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=cl)
        ref = conv_ops._miopen_bwd(gy, x, w, 1, p, (True, False, False))[0]
        bad = 0
        for _ in range(a.runs):
            g = conv_ops._miopen_bwd(gy, x, w, 1, p, (True, False, False))[0]
            bad += int(not torch.equal(g.view(torch.int16), ref.view(torch.int16)))
        print("miopen bf16 dgrad x%s w%s: %d of %d runs differ" % (tuple(x.shape), tuple(w.shape), bad, a.runs),
              flush=True)
        if k == 1:
            m0 = conv_ops._dgrad_mm_bf16(gy, w)
            badm = sum(int(not torch.equal(conv_ops._dgrad_mm_bf16(gy, w).view(torch.int16), m0.view(torch.int16)))
                       for _ in range(a.runs))
            d = (m0.float() - ref.float()).abs().max()
            print("  gemm form: %d of %d runs differ; max |gemm - miopen| %.3e" % (badm, a.runs, float(d)), flush=True)


if __name__ == "__main__":
    main()
