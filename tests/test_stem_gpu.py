"""Stem convolution forward and weight gradient (stem_ops / md2_stem_fwd, md2_stem_wgrad,
split-bf16 MFMA) vs MIOpen's conv2d forward / backward on the same inputs, against an
fp64 reference (fixed-order fp32 sums over 147-294 taps / up to 92k pixels: ours must be
no worse than 2x MIOpen's drift)."""
import pytest
import torch

from monodepth2_amd import stem_ops
from monodepth2_amd.stem_ops import stem_conv, supports_stem

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _enabled(monkeypatch):
    monkeypatch.setattr(stem_ops, "ENABLED", True)
    monkeypatch.setattr(stem_ops, "FWD_ENABLED", True)


def _no_worse(ours, ref, exact, rel=1e-6):
    e_ours = (ours.double() - exact).abs().max().item()
    e_ref = (ref.double() - exact).abs().max().item()
    assert e_ours <= 2 * e_ref + rel * exact.abs().max().item() + 1e-6, (e_ours, e_ref)


@pytest.mark.parametrize("B,C,H,W", [(2, 3, 64, 128), (3, 6, 30, 50), (1, 9, 17, 23), (2, 3, 192, 640),
                                     (1, 6, 7, 9), (2, 6, 192, 640), (1, 6, 9, 300)])
@pytest.mark.parametrize("w_cl", [True, False])
def test_stem_wgrad_matches_conv_backward(B, C, H, W, w_cl):
    torch.manual_seed(7)
    CL = torch.channels_last
    conv = torch.nn.Conv2d(C, 64, 7, 2, 3, bias=False).cuda()
    if w_cl:
        conv = conv.to(memory_format=CL)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    assert supports_stem(conv, x)
    y = stem_conv(conv, x)
    ref = torch.nn.functional.conv2d(x, conv.weight, None, 2, 3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=CL)
    y64 = torch.nn.functional.conv2d(x.double(), conv.weight.double(), None, 2, 3)
    if C == 9:
        assert torch.equal(y, ref)                  # the forward is MIOpen's for three frames
    else:
        _no_worse(y.detach(), ref.detach(), y64.detach())
    g = torch.randn_like(ref).contiguous(memory_format=CL)
    assert y.grad_fn is not None and "StemConv" in type(y.grad_fn).__name__
    gw, = torch.autograd.grad(y, conv.weight, g)
    gwr, = torch.autograd.grad(ref, conv.weight, g)
    assert gw.shape == gwr.shape and gw.is_contiguous(memory_format=CL) == w_cl
    gw64, = torch.autograd.grad(torch.nn.functional.conv2d(x.double(), conv.weight.double(), None, 2, 3),
                                conv.weight, g.double())
    _no_worse(gw, gwr, gw64)


@pytest.mark.parametrize("B,C,H,W", [(2, 6, 192, 640), (1, 3, 1, 1), (2, 3, 5, 130), (1, 6, 64, 200)])
def test_stem_fwd_without_grad(B, C, H, W):
    """The eval / no-grad forward runs md2_stem_fwd too: ragged widths (a partial last
    64-pixel tile), single-pixel images, rows where most of the 7x7 window is padding."""
    torch.manual_seed(3)
    CL = torch.channels_last
    conv = torch.nn.Conv2d(C, 64, 7, 2, 3, bias=False).cuda()
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    with torch.no_grad():
        y = stem_conv(conv, x)
        ref = torch.nn.functional.conv2d(x, conv.weight, None, 2, 3)
        y64 = torch.nn.functional.conv2d(x.double(), conv.weight.double(), None, 2, 3)
    assert y.shape == ref.shape
    _no_worse(y, ref, y64)


def test_stem_falls_back_when_the_input_needs_a_gradient():
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(1, 3, 20, 24, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    assert not supports_stem(conv, x)
    y = stem_conv(conv, x)
    gx, = torch.autograd.grad(y.sum(), x)
    assert gx.shape == x.shape


@pytest.mark.parametrize("B,C,H,W", [(2, 3, 64, 128), (3, 6, 30, 50), (1, 6, 7, 9), (2, 6, 192, 640),
                                     (1, 6, 9, 300), (2, 3, 192, 640)])
@pytest.mark.parametrize("w_cl", [True, False])
def test_stem_wgrad_bf16_operands_bitwise_the_fp32_path(B, C, H, W, w_cl):
    """md2_stem_wgrad with MD2_STEM_BF16 (ABI 23: x and grad_y as bf16, config C5's
    autocast stem) equals the fp32 path on the same values cast up, bit for bit: a bf16
    value splits into itself and two zero planes, whose five products add exact zeros in
    the same accumulation order."""
    import ctypes
    from monodepth2_amd import _lib
    torch.manual_seed(11)
    CL = torch.channels_last
    xb = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    gb = torch.randn(B, 64, Ho, Wo, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    L = _lib.lib()
    fmt = CL if w_cl else torch.contiguous_format

    def run(x, g, flags):
        d = _lib.StemDesc(B, C, H, W, flags | (_lib.STEM_WEIGHT_CL if w_cl else 0))
        gw = torch.empty(64, C, 7, 7, device="cuda", memory_format=fmt)
        ws = torch.empty(L.md2_stem_wgrad_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device="cuda")
        _lib.check(L.md2_stem_wgrad(ctypes.byref(d), x.data_ptr(), g.data_ptr(), gw.data_ptr(), ws.data_ptr(),
                                    _lib.stream(x.device)), "md2_stem_wgrad")
        return gw

    want = run(xb.float().contiguous(memory_format=CL), gb.float().contiguous(memory_format=CL), 0)
    got = run(xb, gb, _lib.STEM_BF16)
    assert torch.equal(got, want)


@pytest.mark.parametrize("B,C,H,W", [(2, 3, 64, 128), (3, 6, 30, 50), (1, 6, 7, 9), (2, 6, 192, 640),
                                     (1, 3, 9, 300), (2, 3, 192, 640), (1, 3, 1, 1)])
@pytest.mark.parametrize("w_cl", [True, False])
def test_stem_fwd_bf16_operands(B, C, H, W, w_cl):
    """md2_stem_fwd with MD2_STEM_BF16 (ABI 23): the bf16 autocast stem — bf16 x, the
    weight rounded to bf16, fp32 accumulation, bf16 y — against an fp64 convolution of the
    same bf16 operands: every element within one bf16 ulp (+ 1e-6 max|ref|) of it, relative
    L2 within 2.5e-3 (the final rounding), bitwise repeatable."""
    torch.manual_seed(13)
    CL = torch.channels_last
    w = (torch.randn(64, C, 7, 7, device="cuda") / (49 * C) ** 0.5)
    w = w.contiguous(memory_format=CL) if w_cl else w.contiguous()
    xb = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    y = stem_ops._fwd_bf16(xb, w)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
    ref = torch.nn.functional.conv2d(xb.double(), w.to(torch.bfloat16).double(), None, 2, 3)
    g = y.double()
    rel = float((g - ref).norm() / ref.norm().clamp_min(1e-30))
    assert rel <= 2.5e-3, rel
    ulp = ref.abs() * 2.0 ** -7 + 1e-6 * ref.abs().max()
    assert int(((g - ref).abs() > ulp).sum()) == 0, float((g - ref).abs().max())
    assert torch.equal(y, stem_ops._fwd_bf16(xb, w))
