"""bf16 autocast convolutions on the per-tap GEMMs (MD2_CONV_BF16, ABI 22; config C5).

A bf16 autocast convolution multiplies bf16 operands — the activations cast to bf16 and
the fp32 weight rounded to bf16 — and returns bf16.  The kernels form every product
exactly in the MFMA's f32 accumulator and round once at the end, so against an fp64
convolution of the same bf16 operands the only error is the f32 accumulation (~1e-7)
plus the final rounding to bf16 (at most half a bf16 ulp, 2^-9 relative).  Bars:
relative L2 <= 2.5e-3 (a uniformly distributed half-ulp rounding gives ~1.6e-3) and no
element further than one bf16 ulp + 1e-6 max|ref| from the rounded fp64 value.  The
weight gradient leaves as fp32 values rounded to bf16 (autocast's cast backward), held
to the same bars.  Every variant is bitwise repeatable, and MIOpen's bf16 convolution of
the same operands (F.conv2d under autocast) is within the same bar of the fp64 value.
"""
import pytest
import torch
import torch.nn.functional as F

from monodepth2_amd import conv_ops

pytestmark = pytest.mark.gpu

CL = torch.channels_last
BF = conv_ops.BF

SHAPES = [  # (B, Cin, Cout, k, stride, pad, H, W)
    (2, 64, 64, 3, 1, 1, 24, 40),      # ResNet layer1
    (3, 128, 128, 3, 1, 1, 12, 20),    # 128-wide tiles
    (2, 256, 256, 3, 1, 1, 6, 10),     # deep layer: K split
    (2, 64, 128, 3, 2, 1, 24, 40),     # stage entry, stride 2 (dgrad: parity classes)
    (2, 64, 128, 1, 2, 0, 23, 39),     # downsample shortcut, odd sizes: three tapless classes
    (2, 64, 128, 3, 2, 1, 23, 39),     # stride 2 on odd sizes: unequal parity classes
    (2, 96, 64, 3, 1, 0, 18, 34),      # decoder conv on a padded input
    (2, 32, 16, 3, 1, 0, 18, 34),      # decoder 16-channel layer: 16-wide tile, flattened K
    (2, 16, 16, 3, 1, 0, 18, 34),      # 16 -> 16: flattened K on both sides
    (4, 256, 12, 1, 1, 0, 6, 20),      # pose decoder pose_2: 12 outputs
]


def _rne(t):
    return t.to(torch.bfloat16)


def _check(got, ref64, what):
    """got (bf16 or bf16-valued fp32) against the fp64 value of the same operands"""
    g = got.double()
    r = ref64
    rel = float((g - r).norm() / r.norm().clamp_min(1e-30))
    assert rel <= 2.5e-3, (what, rel)
    ulp = r.abs() * 2.0 ** -7 + 1e-6 * r.abs().max()   # one bf16 ulp (8 significant bits)
    bad = int(((g - r).abs() > ulp).sum())
    assert bad == 0, (what, bad, float((g - r).abs().max()))


def _case(B, C, N, k, s, p, H, W, seed=0):
    torch.manual_seed(seed + B * 1000 + C + N + k + s + H)
    x = _rne(torch.randn(B, C, H, W, device="cuda")).contiguous(memory_format=CL)
    w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
    return x, w


@pytest.mark.parametrize("B,C,N,k,s,p,H,W", SHAPES)
def test_bf16_kernels_match_fp64(B, C, N, k, s, p, H, W):
    x, w = _case(B, C, N, k, s, p, H, W)
    wb = _rne(w)
    x64, w64 = x.double(), wb.double()
    y64 = F.conv2d(x64, w64, None, s, p)
    gy = _rne(torch.randn(y64.shape, device="cuda")).contiguous(memory_format=CL)
    gx64, gw64 = torch.ops.aten.convolution_backward(gy.double(), x64, w64, None, (s, s), (p, p), (1, 1), False,
                                                     (0, 0), 1, (True, True, False))[:2]
    pf, pd = conv_ops._bf16_weights(x, w, s, p, N % 8 == 0 and (s == 1 or N >= 32))
    assert torch.equal(pf.view(N, k, k, C).permute(0, 3, 1, 2), wb)   # the weight rounded to nearest even
    flags = list(conv_ops._bf_flags(N, C, k, s)[0])
    if C % 8 == 0:
        for f in flags:
            y = conv_ops._fwd_bf(x, w, pf, s, p, f)
            assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
            _check(y, y64, ("fwd", f))
            assert torch.equal(y, conv_ops._fwd_bf(x, w, pf, s, p, f)), ("fwd repeat", f)
    if pd is not None:   # stride 2: the four output-parity classes, per-class launches or one
        dflags = list(conv_ops._bf_flags(C, N, k, 1)[0]) if s == 1 else [BF, BF | conv_ops.S2_ONE]
        for f in dflags:
            gx = conv_ops._dgrad_bf(gy, x, w, pd, p, f, s)
            assert gx.dtype == torch.bfloat16
            _check(gx, gx64, ("dgrad", f))
            assert torch.equal(gx, conv_ops._dgrad_bf(gy, x, w, pd, p, f, s)), ("dgrad repeat", f)
    wflags = [BF] + ([BF | conv_ops.PATCH] if (k == 3 and s == 1) else []) + \
        ([BF | conv_ops.WS | conv_ops.BM256] if N > 64 else [])   # per-tap / patch-staged / 256-wide
    for f in wflags:
        gw = conv_ops._wgrad_bf(gy, x, w, s, p, f)
        assert gw.dtype == torch.float32 and torch.equal(gw, gw.to(torch.bfloat16).float())   # bf16 values
        _check(gw, gw64, ("wgrad", f))
        assert torch.equal(gw, conv_ops._wgrad_bf(gy, x, w, s, p, f)), ("wgrad repeat", f)
    # MIOpen's bf16 convolution of the same operands, for scale (its own summation order)
    ym = F.conv2d(x, wb, None, s, p).double()
    assert float((ym - y64).norm() / y64.norm()) <= 5e-3


@pytest.mark.parametrize("B,C,N,k,s,p,H,W", [SHAPES[0], SHAPES[3], SHAPES[6], SHAPES[8], SHAPES[9]])
def test_bf16_autocast_conv_through_conv_ops(B, C, N, k, s, p, H, W, monkeypatch):
    """conv_ops.conv2d under bf16 autocast: the output and both gradients of the
    production path (autotuned against MIOpen; a non-repeatable candidate never kept)
    within the bars of the fp64 value of autocast's operands, and bitwise repeatable."""
    monkeypatch.setattr(conv_ops, "_choice", {})
    conv = torch.nn.Conv2d(C, N, k, s, p, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL).requires_grad_(True)

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = conv_ops.conv2d(conv, x)
        assert y.dtype == torch.bfloat16
        g = ((torch.arange(y.numel(), device="cuda").view_as(y) % 7) - 3).to(y.dtype)
        gx, gw = torch.autograd.grad(y, [x, conv.weight], g)
        return y, g, gx, gw

    y, g, gx, gw = run()
    y2, _, gx2, gw2 = run()
    assert torch.equal(y, y2) and torch.equal(gx, gx2) and torch.equal(gw, gw2)
    x64, w64 = _rne(x.detach()).double(), _rne(conv.weight.detach()).double()
    y64 = F.conv2d(x64, w64, None, s, p)
    gx64, gw64 = torch.ops.aten.convolution_backward(g.double(), x64, w64, None, (s, s), (p, p), (1, 1), False,
                                                     (0, 0), 1, (True, True, False))[:2]
    _check(y, y64, "fwd")
    _check(gx, gx64, "dgrad")   # the cast's backward: the bf16 gradient as fp32
    _check(gw, gw64, "wgrad")
    assert "fwd_bf16" in {k[0] for k in conv_ops._choice}
    if k == 1 and N % 8:   # pose_2: the input gradient on the GEMM form (_dgrad_mm_bf16), not timed
        assert ("dgrad_bf16", (B, C, H, W), (N, C, k, k), s, p) not in conv_ops._choice


@pytest.mark.parametrize("B,C,N,p,H,W", [(2, 16, 16, 0, 18, 34), (2, 32, 16, 0, 18, 34), (2, 16, 32, 0, 18, 34),
                                         (3, 16, 16, 1, 20, 70), (2, 32, 16, 1, 9, 11)])
def test_bf16_direct_16_channel_forms(B, C, N, p, H, W):
    """md2_conv_direct / md2_conv_wgrad_direct with MD2_CONV_X6 | MD2_CONV_BF16 (the
    decoder's 16-channel full-resolution layers under autocast): forward, input gradient
    (roles swapped, flipped weight) and weight gradient within the bars above of the fp64
    convolution of the same bf16 operands; bitwise repeatable."""
    from monodepth2_amd.conv_ops import _direct_dgrad, _direct_fwd, _direct_ok, _direct_wgrad, X6
    x, w = _case(B, C, N, 3, 1, p, H, W)
    wb = _rne(w)
    x64, w64 = x.double(), wb.double()
    if _direct_ok(C, N, 3, 1):
        y = _direct_fwd(x, w, p, X6 | BF)
        assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
        _check(y, F.conv2d(x64, w64, None, 1, p), "fwd")
        assert torch.equal(y, _direct_fwd(x, w, p, X6 | BF))
    y64 = F.conv2d(x64, w64, None, 1, p)
    gy = _rne(torch.randn(y64.shape, device="cuda")).contiguous(memory_format=CL)
    gx64, gw64 = torch.ops.aten.convolution_backward(gy.double(), x64, w64, None, (1, 1), (p, p), (1, 1), False,
                                                     (0, 0), 1, (True, True, False))[:2]
    if _direct_ok(N, C, 3, 1):
        gx = _direct_dgrad(gy, w, p, X6 | BF)
        assert gx.dtype == torch.bfloat16
        _check(gx, gx64, "dgrad")
        assert torch.equal(gx, _direct_dgrad(gy, w, p, X6 | BF))
    if _direct_ok(C, N, 3, 1) and N == 16:
        gw = _direct_wgrad(gy, x, w, p, X6 | BF)
        _check(gw.to(torch.bfloat16).float(), gw64, "wgrad")
        assert torch.equal(gw, _direct_wgrad(gy, x, w, p, X6 | BF))
