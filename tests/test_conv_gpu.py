"""f32 MFMA implicit-GEMM convolutions (csrc/conv.hip via conv_ops) vs MIOpen
(F.conv2d, fp32) on the encoder / decoder shapes: outputs and gradients.

f32 MFMA is an exact f32 fma chain, so the two differ only in summation order:
the bar is 2e-5 of the output's magnitude (forward) and 1e-4 (gradients)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from monodepth2_amd import _lib, conv_ops

pytestmark = pytest.mark.gpu

CL = torch.channels_last

SHAPES = [  # (B, Cin, Cout, k, stride, pad, H, W)
    (2, 64, 64, 3, 1, 1, 24, 40),      # ResNet layer1 conv
    (3, 128, 128, 3, 1, 1, 12, 20),    # 128x128 tile
    (2, 64, 128, 3, 2, 1, 24, 40),     # stage-entry conv, stride 2
    (2, 64, 128, 1, 2, 0, 24, 40),     # downsample shortcut
    (2, 256, 256, 3, 1, 1, 6, 10),     # deep layer: K split
    (2, 512, 512, 3, 1, 1, 3, 5),      # layer4 at 96x320: K split, M tail
    (2, 96, 64, 3, 1, 0, 18, 34),      # decoder conv on a padded input (pad 0), C = 3 chunks
    (1, 32, 64, 3, 1, 1, 7, 9),        # odd sizes, M not a tile multiple
    (2, 64, 128, 3, 2, 1, 23, 39),     # stride 2 on odd sizes: unequal parity classes
    (2, 64, 128, 1, 2, 0, 23, 39),     # 1x1 stride 2 on odd sizes: three tapless classes
]


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.fixture(autouse=True)
def _mfma_always(monkeypatch):
    """These tests check the MFMA kernels themselves: no per-shape fallback to MIOpen."""
    monkeypatch.setattr(conv_ops, "AUTOTUNE", False)


@pytest.mark.parametrize("B,C,N,k,s,p,H,W", SHAPES)
def test_conv_matches_miopen(B, C, N, k, s, p, H, W):
    torch.manual_seed(B * 1000 + C + N + k + s + H)
    conv = torch.nn.Conv2d(C, N, k, s, p, bias=False).cuda().to(memory_format=CL)
    ref = torch.nn.Conv2d(C, N, k, s, p, bias=False).cuda().to(memory_format=CL)
    ref.weight.data.copy_(conv.weight.data)
    x0 = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    x = x0.clone().requires_grad_(True)
    xr = x0.clone().requires_grad_(True)
    assert conv_ops.supports(conv, x)
    y = conv_ops.conv2d(conv, x)
    yr = ref(xr)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 2e-5
    g = torch.randn_like(yr)
    gx, gw = torch.autograd.grad(y, [x, conv.weight], g)
    gxr, gwr = torch.autograd.grad(yr, [xr, ref.weight], g)
    assert _rel(gx, gxr) < 1e-4
    assert _rel(gw, gwr) < 1e-4


def test_autotune_keeps_a_choice_per_shape(monkeypatch):
    """With AUTOTUNE the first call of a shape times the MFMA kernel against MIOpen
    and caches the winner; either way the result is the convolution."""
    monkeypatch.setattr(conv_ops, "AUTOTUNE", True)
    monkeypatch.setattr(conv_ops, "_choice", {})
    conv = torch.nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(2, 64, 24, 40, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    y = conv_ops.conv2d(conv, x)
    y.backward(torch.ones_like(y))
    assert {k[0] for k in conv_ops._choice} == {"fwd", "dgrad", "wgrad"}
    assert _rel(y, F.conv2d(x, conv.weight, padding=1)) < 2e-5


def test_conv_tile_and_split_variants_agree():
    """The 128x64 / 128x128 tiles and the K split (partials summed in split order)
    give the same result up to rounding; each run is bitwise deterministic."""
    torch.manual_seed(7)
    B, C, N, H, W = 2, 256, 256, 12, 20
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(N, C, 3, 3, device="cuda").contiguous(memory_format=CL) / 48
    outs = {}
    for flags in (0, _lib.CONV_TILE_N64, _lib.CONV_TILE_N32, _lib.CONV_NO_SPLIT,
                  _lib.CONV_TILE_N64 | _lib.CONV_NO_SPLIT):
        d = _lib.ConvDesc(B, H, W, C, N, 3, 3, 1, 1, flags)
        L = _lib.lib()
        ws = torch.empty(max(L.md2_conv_workspace_bytes(ctypes.byref(d)), 4), dtype=torch.uint8, device="cuda")
        res = []
        for _ in range(2):
            y = torch.empty(B, N, H, W, device="cuda", memory_format=CL)
            _lib.check(L.md2_conv_fwd(ctypes.byref(d), x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream), "md2_conv_fwd")
            res.append(y)
        assert torch.equal(res[0], res[1])
        outs[flags] = res[0]
    ref = F.conv2d(x, w, padding=1)
    for y in outs.values():
        assert _rel(y, ref) < 2e-5


def test_conv_rejects_unsupported_shapes():
    d = _lib.ConvDesc(1, 8, 8, 6, 64, 3, 3, 1, 1, 0)   # in_channels not a multiple of 4
    assert _lib.lib().md2_conv_fwd(ctypes.byref(d), 1, 1, 1, 1, None) == -1
    d = _lib.ConvDesc(1, 8, 8, 8, 64, 3, 3, 2, 1, 0)   # the input gradient is stride 1 only
    assert _lib.lib().md2_conv_dgrad(ctypes.byref(d), 1, 1, 1, 1, None) == -1


def test_encoder_on_mfma_convs_matches_miopen():
    """Whole ResNet-18 encoder, training mode: MFMA convs vs MIOpen convs (same fused
    BatchNorm), features and every parameter gradient."""
    import copy
    from monodepth2_amd import networks
    torch.manual_seed(0)
    enc = networks.ResnetEncoder(18, False).cuda().to(memory_format=CL)
    ref = copy.deepcopy(enc)
    img = torch.rand(2, 3, 64, 128, device="cuda")

    def run(e, on):
        conv_ops.ENABLED = on
        try:
            feats = e(img)
        finally:
            conv_ops.ENABLED = True
        loss = sum((f * (i + 1)).mean() for i, f in enumerate(feats))
        return feats, torch.autograd.grad(loss, list(e.parameters()), allow_unused=True)

    fa, ga = run(enc, True)
    fb, gb = run(ref, False)
    for a, b in zip(fa, fb):
        assert float((a - b).norm() / b.norm()) < 1e-5
    for a, b in zip(ga, gb):
        if b is not None:
            assert float((a - b).norm() / (b.norm() + 1e-12)) < 1e-3


@pytest.mark.parametrize("B,C,N,k,s,p,H,W", SHAPES + [(2, 16, 16, 3, 1, 0, 20, 34), (2, 32, 16, 3, 1, 0, 12, 18),
                                                      (2, 96, 32, 3, 1, 0, 10, 12), (2, 64, 32, 3, 1, 0, 9, 11)])
def test_conv_abi_dgrad_wgrad(B, C, N, k, s, p, H, W):
    """md2_conv_dgrad / md2_conv_wgrad directly (every tile width, K split on),
    including the decoder's narrow full-resolution convs (16 / 32 channels)."""
    torch.manual_seed(3 + C + N + H)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
    y = F.conv2d(x, w, stride=s, padding=p)
    gy = torch.randn_like(y).contiguous(memory_format=CL)
    gx_ref, gw_ref, _ = torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                                            (True, True, False))
    L = _lib.lib()
    d = _lib.ConvDesc(B, H, W, C, N, k, k, s, p, 0)
    ws = torch.empty(max(L.md2_conv_workspace_bytes(ctypes.byref(d)), 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    yo = torch.empty_like(y, memory_format=CL)
    _lib.check(L.md2_conv_fwd(ctypes.byref(d), x.data_ptr(), w.data_ptr(), yo.data_ptr(), ws.data_ptr(), st), "fwd")
    assert _rel(yo, y) < 2e-5
    gw = torch.empty_like(w, memory_format=CL)
    _lib.check(L.md2_conv_wgrad(ctypes.byref(d), x.data_ptr(), gy.data_ptr(), gw.data_ptr(), ws.data_ptr(), st),
               "wgrad")
    assert _rel(gw, gw_ref) < 1e-4
    if s == 1:
        gx = torch.empty_like(x, memory_format=CL)
        _lib.check(L.md2_conv_dgrad(ctypes.byref(d), gy.data_ptr(), w.data_ptr(), gx.data_ptr(), ws.data_ptr(), st),
                   "dgrad")
        assert _rel(gx, gx_ref) < 1e-4


# x6 variants: 128 / 256-row tiles, the patch-staged kernel (which run() uses only where
# the shape fits it: 3x3, stride 1, GEMM channels % 32 — elsewhere the flag is inert) and
# the one-launch stride-2 input gradient (inert at stride 1)
XFLAGS = (conv_ops.X6, conv_ops.X6 | conv_ops.BM256, conv_ops.X6 | conv_ops.PATCH,
          conv_ops.X6 | conv_ops.PATCH | conv_ops.BM256, conv_ops.X6 | conv_ops.S2_ONE,
          conv_ops.X6 | conv_ops.S2_ONE | conv_ops.BM256, conv_ops.X6 | conv_ops.WS,
          conv_ops.X6 | conv_ops.WS | conv_ops.BM256)


# + the decoder's narrow layers: 16 output channels take the 16x16x32 MFMA tile (its own
# LDS slot swizzle), 32 the 128 x 32 one
@pytest.mark.parametrize("B,C,N,k,s,p,H,W", [sh for sh in SHAPES if sh[1] % 8 == 0 and sh[2] % 8 == 0] +
                         [(2, 16, 16, 3, 1, 0, 20, 34), (2, 32, 16, 3, 1, 0, 12, 18), (2, 96, 32, 3, 1, 0, 10, 12)])
def test_x6_split_bf16_is_f32_class(B, C, N, k, s, p, H, W):
    """The split-bf16 path (MD2_CONV_X6: exact three-plane split, six bf16 MFMA
    products, f32 accumulation) against an fp64 reference: its error is of the order
    of MIOpen's own f32 error (within 3x of it, and below 2e-6 of the output's
    magnitude), forward, input and weight gradient — f32-class, not reduced precision."""
    torch.manual_seed(11 + C + N + H)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), None, s, p)
    y_mi = F.conv2d(x, w, None, s, p).double().cpu()
    e_mi = _rel(y_mi, ref)
    for fl in XFLAGS:
        e_x6 = _rel(conv_ops._fwd(x, w, s, p, fl).double().cpu(), ref)
        assert e_x6 < max(3 * e_mi, 1e-7) and e_x6 < 2e-6, (fl, e_x6, e_mi)
    if s == 1 or conv_ops._x6_s2_ok(x, w, s):   # stride 2: four parity-class GEMMs
        gy = torch.randn(ref.shape, device="cuda").contiguous(memory_format=CL)
        gref = torch.ops.aten.convolution_backward(gy.double().cpu(), x.double().cpu(), w.double().cpu(), None, (s, s),
                                                   (p, p), (1, 1), False, (0, 0), 1, (True, False, False))[0]
        g_mi = torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                                   (True, False, False))[0].double().cpu()
        e_mi = _rel(g_mi, gref)
        for fl in XFLAGS:
            e_x6 = _rel(conv_ops._dgrad(gy, x, w, p, fl, s).double().cpu(), gref)
            assert e_x6 < max(3 * e_mi, 1e-7) and e_x6 < 2e-6, (fl, s, e_x6, e_mi)
        if s == 2:   # one GEMM over every tap + md2_conv_col2im's gather
            for fl in (conv_ops.X6, conv_ops.X6 | conv_ops.BM256):
                e_col = _rel(conv_ops._dgrad_col(gy, x, w, s, p, fl).double().cpu(), gref)
                assert e_col < max(3 * e_mi, 1e-7) and e_col < 2e-6, (fl, e_col, e_mi)
    gy = torch.randn(ref.shape, device="cuda").contiguous(memory_format=CL)
    wref = torch.ops.aten.convolution_backward(gy.double().cpu(), x.double().cpu(), w.double().cpu(), None, (s, s),
                                               (p, p), (1, 1), False, (0, 0), 1, (False, True, False))[1]
    w_x6 = conv_ops._wgrad(gy, x, w, s, p, conv_ops.X6).double().cpu()
    w_mi = torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                               (False, True, False))[1].double().cpu()
    e_x6, e_mi = _rel(w_x6, wref), _rel(w_mi, wref)
    assert e_x6 < max(3 * e_mi, 1e-7) and e_x6 < 2e-6, ("wgrad", e_x6, e_mi)


@pytest.mark.parametrize("B,C,N,k,s,p,H,W", [(2, 64, 128, 3, 1, 1, 24, 40), (3, 128, 128, 3, 1, 1, 12, 20),
                                             (2, 256, 256, 3, 1, 1, 6, 10), (2, 512, 512, 3, 1, 1, 3, 5),
                                             (2, 64, 128, 3, 2, 1, 23, 39), (2, 64, 128, 1, 2, 0, 24, 40),
                                             (1, 96, 136, 3, 1, 1, 7, 9), (2, 512, 256, 3, 1, 1, 6, 20)])
def test_x6_warp_specialised_is_bitwise_the_per_tap_kernel(B, C, N, k, s, p, H, W):
    """MD2_CONV_WS (4 MFMA waves + 4 staging waves per block) computes the same products
    in the same order per output as conv_x6_kernel with the same tile height: forward and
    stride-1 input gradient bitwise equal, K splits, M / N tails, stride 2 included.  The
    weight gradient's warp-specialised kernel (conv_x6wws_kernel) likewise against
    conv_x6_wgrad_kernel<128>, with and without its K split and pixel walk (Wo % 4)."""
    torch.manual_seed(3 + C + N + H)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
    for extra in (0, conv_ops.BM256, conv_ops.NO_SPLIT, conv_ops.BM256 | conv_ops.NO_SPLIT):
        base = conv_ops.X6 | extra
        assert torch.equal(conv_ops._fwd(x, w, s, p, base | conv_ops.WS), conv_ops._fwd(x, w, s, p, base)), extra
        if s == 1:
            gy = torch.randn(conv_ops._fwd(x, w, s, p, base).shape, device="cuda").contiguous(memory_format=CL)
            assert torch.equal(conv_ops._dgrad(gy, x, w, p, base | conv_ops.WS), conv_ops._dgrad(gy, x, w, p, base)), extra
    gy = torch.randn(conv_ops._fwd(x, w, s, p, conv_ops.X6).shape, device="cuda").contiguous(memory_format=CL)
    for extra in (0, conv_ops.NO_SPLIT):
        base = conv_ops.X6 | extra
        gw = conv_ops._wgrad(gy, x, w, s, p, base | conv_ops.WS)
        assert torch.equal(gw, conv_ops._wgrad(gy, x, w, s, p, base)), ("wgrad", extra)
        assert torch.equal(gw, conv_ops._wgrad(gy, x, w, s, p, base | conv_ops.WS)), ("wgrad repeat", extra)


@pytest.mark.parametrize("B,C,N,k,s,p,H,W", [(2, 128, 128, 3, 1, 1, 24, 40), (2, 256, 256, 3, 1, 1, 12, 20),
                                             (2, 64, 128, 3, 2, 1, 23, 39), (2, 64, 128, 1, 2, 0, 24, 40),
                                             (1, 96, 136, 3, 1, 1, 7, 9), (2, 512, 256, 3, 1, 0, 8, 22),
                                             (12, 128, 128, 3, 1, 1, 24, 80)])
def test_x6_wgrad_256_wide_tile_is_f32_class(B, C, N, k, s, p, H, W):
    """The weight gradient's 256-wide warp-specialised tile (MD2_CONV_WS | MD2_CONV_BM256:
    two taps of a 128-channel layer per block, one accumulation level over K splits of at
    most 64 chunks) against fp64: within 3x MIOpen's f32 error and below 2e-6, with and
    without the split model's choice (NO_SPLIT still splits past 64 chunks), M / N tails,
    stride 2, the pixel walk off (Wo % 4); bitwise repeatable."""
    torch.manual_seed(5 + C + N + H)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, k, k, device="cuda") / (C * k * k) ** 0.5).contiguous(memory_format=CL)
    gy = torch.randn(F.conv2d(x, w, None, s, p).shape, device="cuda").contiguous(memory_format=CL)
    wref = torch.ops.aten.convolution_backward(gy.double().cpu(), x.double().cpu(), w.double().cpu(), None, (s, s),
                                               (p, p), (1, 1), False, (0, 0), 1, (False, True, False))[1]
    w_mi = torch.ops.aten.convolution_backward(gy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                               (False, True, False))[1].double().cpu()
    e_mi = _rel(w_mi, wref)
    for extra in (0, conv_ops.NO_SPLIT):
        fl = conv_ops.X6 | conv_ops.WS | conv_ops.BM256 | extra
        gw = conv_ops._wgrad(gy, x, w, s, p, fl)
        e = _rel(gw.double().cpu(), wref)
        assert e < max(3 * e_mi, 1e-7) and e < 2e-6, (extra, e, e_mi)
        assert torch.equal(gw, conv_ops._wgrad(gy, x, w, s, p, fl)), ("repeat", extra)


def test_x6_presplit_planes_match_in_call_split():
    """md2_conv_split_weights (both layouts in one pass) + MD2_CONV_PRESPLIT gives
    bitwise the result of the x6 calls that split the weight themselves."""
    torch.manual_seed(5)
    B, C, N, H, W = 2, 64, 128, 12, 20
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / 24).contiguous(memory_format=CL)
    gy = torch.randn(B, N, H, W, device="cuda").contiguous(memory_format=CL)
    pf, pd = conv_ops._split_weights(x, w, 1, 1, True)
    for fl in (conv_ops.X6, conv_ops.X6 | conv_ops.BM256):
        assert torch.equal(conv_ops._fwd_planes(x, w, pf, 1, 1, fl), conv_ops._fwd(x, w, 1, 1, fl))
        assert torch.equal(conv_ops._dgrad_planes(gy, x, w, pd, 1, fl), conv_ops._dgrad(gy, x, w, 1, fl))
    # stride 2 (parity classes) reads the same flipped planes
    gy2 = torch.randn(B, N, H // 2, W // 2, device="cuda").contiguous(memory_format=CL)
    pf2, pd2 = conv_ops._split_weights(x, w, 2, 1, True)
    assert torch.equal(conv_ops._dgrad_planes(gy2, x, w, pd2, 1, conv_ops.X6, 2), conv_ops._dgrad(gy2, x, w, 1, conv_ops.X6, 2))


def test_plane_bank_refresh_matches_per_call_split():
    """conv_ops.PlaneBank: one md2_conv_split_weights_multi launch re-splits every
    registered weight (3x3 / 1x1, with and without input-gradient planes, channel
    counts that are not multiples of 32) into bitwise the planes of the per-call
    split; outside the step window nothing is handed out."""
    torch.manual_seed(6)
    bank = conv_ops.PlaneBank()
    shapes = [(64, 64, 3, 1, True), (128, 64, 1, 2, False), (40, 24, 3, 1, True), (256, 128, 3, 2, True),
              (16, 8, 1, 1, False)]
    ws, xs = [], []
    for N, C, k, s, dg in shapes:
        xs.append(torch.randn(1, C, 8, 8, device="cuda").contiguous(memory_format=CL))
        ws.append(torch.randn(N, C, k, k, device="cuda").contiguous(memory_format=CL))
    assert bank.planes(xs[0], ws[0], 1, 1, True) is None   # window closed
    bank.begin_step(torch.device("cuda", 0))
    for x, w, (N, C, k, s, dg) in zip(xs, ws, shapes):
        pf, pd = bank.planes(x, w, s, k // 2, dg)
        assert (pd is not None) == dg
    bank.end_step()
    with torch.no_grad():   # the optimizer moves the weights
        for w in ws:
            w.mul_(1.5).add_(0.01)
    bank.begin_step(torch.device("cuda", 0))
    assert not bank.dirty and bank.total_blocks > 0
    for x, w, (N, C, k, s, dg) in zip(xs, ws, shapes):
        pf, pd = bank.planes(x, w, s, k // 2, dg)
        rf, rd = conv_ops._split_weights(x, w, s, k // 2, dg)
        assert torch.equal(pf, rf)
        assert (pd is None and rd is None) or torch.equal(pd, rd)
    bank.end_step()


def test_plane_bank_column_planes(monkeypatch):
    """PlaneBank.col_planes: the strided input gradient's column operand ([kh][kw][ci][co]
    split planes) refreshed with the step's other planes is bitwise the per-call permute
    + split, and _dgrad_col through it returns bitwise the same gradient."""
    torch.manual_seed(7)
    bank = conv_ops.PlaneBank()
    monkeypatch.setattr(conv_ops, "_bank", bank)
    B, C, N, H, W = 2, 64, 128, 24, 40
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = torch.randn(N, C, 3, 3, device="cuda").contiguous(memory_format=CL)
    gy = torch.randn(B, N, H // 2, W // 2, device="cuda").contiguous(memory_format=CL)
    flags = conv_ops.X6
    bank.begin_step(torch.device("cuda", 0))
    assert bank.col_planes(w) is None          # first request: registered, filled from the next refresh
    g0 = conv_ops._dgrad_col(gy, x, w, 2, 1, flags)   # per-call permute + split meanwhile
    assert bank.col_planes(w) is None          # still unfilled in this window
    bank.end_step()
    bank.begin_step(torch.device("cuda", 0))
    pc = bank.col_planes(w)
    assert pc is not None
    wcol = w.permute(2, 3, 1, 0).reshape(9 * C, N, 1, 1).contiguous()
    ref, _ = conv_ops._split_weights(gy, wcol, 1, 0, False)
    assert torch.equal(pc, ref)
    g1 = conv_ops._dgrad_col(gy, x, w, 2, 1, flags)
    bank.end_step()
    assert torch.equal(g0, g1)


@pytest.mark.parametrize("B,C,N,p,H,W", [(2, 16, 16, 0, 20, 34), (2, 32, 16, 0, 12, 18), (2, 16, 32, 1, 9, 13),
                                         (1, 16, 16, 1, 7, 9), (3, 32, 16, 2, 5, 6), (2, 16, 16, 0, 70, 131),
                                         (1, 32, 16, 1, 9, 200)])
@pytest.mark.parametrize("flags", [0, conv_ops.X6], ids=["valu", "x6"])
def test_direct_conv_matches_miopen(B, C, N, p, H, W, flags):
    """md2_conv_direct for the DepthDecoder's 16-output-channel layers — f32 VALU (one
    thread per output pixel) or split-bf16 MFMA (X6, weights in registers, patch planes
    in LDS; partial 4 x 64 tiles at the ragged sizes): forward and input gradient vs
    MIOpen fp32 (f32-class sums in different orders)."""
    torch.manual_seed(B * 10 + C + N + p)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / (9 * C) ** 0.5).contiguous(memory_format=CL)
    y = conv_ops._direct_fwd(x, w, p, flags)
    yr = F.conv2d(x, w, padding=p)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 2e-5
    gy = torch.randn_like(yr).contiguous(memory_format=CL)
    gx = conv_ops._direct_dgrad(gy, w, p, flags)
    gxr = torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (p, p), (1, 1), False, (0, 0), 1,
                                              (True, False, False))[0]
    assert gx.shape == x.shape
    assert _rel(gx, gxr) < 1e-4


def test_direct_conv_rejects_other_shapes():
    d = _lib.ConvDesc(1, 8, 8, 64, 16, 3, 3, 1, 1, 0)   # 64 input channels: not a direct shape
    x = torch.zeros(1, 8, 8, 64, device="cuda")
    assert _lib.lib().md2_conv_direct(ctypes.byref(d), x.data_ptr(), x.data_ptr(), x.data_ptr(), None) != 0


@pytest.mark.parametrize("B,C,p,H,W", [(2, 16, 0, 20, 34), (2, 32, 0, 12, 18), (1, 16, 1, 7, 9), (3, 32, 2, 5, 6),
                                       (4, 16, 0, 66, 70), (2, 32, 1, 37, 150)])
@pytest.mark.parametrize("flags", [0, conv_ops.X6], ids=["valu", "x6"])
def test_direct_wgrad_matches_miopen(B, C, p, H, W, flags):
    """md2_conv_wgrad_direct — f32 VALU or split-bf16 MFMA (X6: transposed LDS reads of
    the staged planes, partial 4 x 64 tiles at the ragged sizes) — per-block partial rows
    summed in block order, vs an fp64 reference (no worse than 3x MIOpen's fp32 drift)
    and bitwise reproducible run to run."""
    torch.manual_seed(B * 10 + C + p + H)
    N = 16
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / (9 * C) ** 0.5).contiguous(memory_format=CL)
    gy = torch.randn_like(F.conv2d(x, w, padding=p)).contiguous(memory_format=CL)
    gw = conv_ops._direct_wgrad(gy, x, w, p, flags)
    gwr = torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (p, p), (1, 1), False, (0, 0), 1,
                                              (False, True, False))[1]
    g64 = torch.ops.aten.convolution_backward(gy.double(), x.double(), w.double(), None, (1, 1), (p, p), (1, 1),
                                              False, (0, 0), 1, (False, True, False))[1]
    assert gw.shape == w.shape and gw.is_contiguous(memory_format=CL)
    assert _rel(gw, gwr) < 1e-4
    assert _rel(gw.double(), g64) <= 3 * _rel(gwr.double(), g64) + 1e-7
    assert torch.equal(gw, conv_ops._direct_wgrad(gy, x, w, p, flags))


PATCH_SHAPES = [  # (B, Cin, Cout, pad, H, W): tile-column choices 64 / 32 / 16, odd tails, K splits
    (2, 64, 64, 1, 24, 80),     # layer-1-like width: 16-column tiles
    (2, 128, 128, 1, 12, 40),   # 64-column tiles with a 24-column tail
    (1, 96, 64, 0, 18, 34),     # decoder conv on a pre-padded input (pad 0; input gradient pad 2)
    (2, 256, 256, 1, 6, 10),    # deep layer: K split over channel chunks
    (3, 32, 32, 1, 7, 9),       # one channel chunk, 32 output columns, odd sizes
    (2, 64, 128, 1, 48, 160),   # wide: 64-column tiles
    (2, 512, 64, 1, 5, 7),      # many chunks, tiny image
]


@pytest.mark.parametrize("B,C,N,p,H,W", PATCH_SHAPES)
def test_x6_patch_kernel_is_f32_class(B, C, N, p, H, W):
    """The patch-staged split-bf16 kernel (MD2_CONV_PATCH: one input patch per 32
    channels for all nine taps) on forward and stride-1 input gradient against fp64:
    f32-class like the per-tap x6 kernel, and within 2e-6 of it."""
    torch.manual_seed(31 + C + N + H + W)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / (C * 9) ** 0.5).contiguous(memory_format=CL)
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), None, 1, p)
    e_mi = _rel(F.conv2d(x, w, None, 1, p).double().cpu(), ref)
    gy = torch.randn(ref.shape, device="cuda").contiguous(memory_format=CL)
    gref = torch.ops.aten.convolution_backward(gy.double().cpu(), x.double().cpu(), w.double().cpu(), None, (1, 1),
                                               (p, p), (1, 1), False, (0, 0), 1, (True, False, False))[0]
    g_mi = torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (p, p), (1, 1), False, (0, 0), 1,
                                               (True, False, False))[0].double().cpu()
    eg_mi = _rel(g_mi, gref)
    base_y = conv_ops._fwd(x, w, 1, p, conv_ops.X6).double().cpu()
    base_g = conv_ops._dgrad(gy, x, w, p, conv_ops.X6).double().cpu()
    for fl in (conv_ops.X6 | conv_ops.PATCH, conv_ops.X6 | conv_ops.PATCH | conv_ops.BM256):
        y = conv_ops._fwd(x, w, 1, p, fl).double().cpu()
        e = _rel(y, ref)
        assert e < max(3 * e_mi, 1e-7) and e < 2e-6, (fl, e, e_mi)
        assert _rel(y, base_y) < 2e-6
        g = conv_ops._dgrad(gy, x, w, p, fl).double().cpu()
        e = _rel(g, gref)
        assert e < max(3 * eg_mi, 1e-7) and e < 2e-6, (fl, e, eg_mi)
        assert _rel(g, base_g) < 2e-6
        assert torch.equal(conv_ops._fwd(x, w, 1, p, fl), conv_ops._fwd(x, w, 1, p, fl))   # deterministic


PATCH_W_SHAPES = [  # (B, Cin, Cout, pad, H, W): segment tails, partial channel groups, Co 16 / 24 / 32 / 128
    (2, 64, 64, 1, 24, 80),     # 80 columns: two full 32-column segments and a 16-column tail
    (1, 96, 32, 0, 18, 34),     # decoder conv on a pre-padded input, Co 32 (32-row tile)
    (2, 16, 16, 1, 20, 70),     # 16 input channels: half a channel group, Co 16
    (3, 32, 32, 2, 7, 9),       # pad 2, one short segment
    (2, 128, 128, 1, 12, 40),   # two row blocks x four channel groups
    (2, 40, 24, 1, 9, 33),      # 40 channels (8 in the second group), Co 24, a 1-column tail
    (4, 64, 64, 1, 48, 160),    # layer-1 shape: many chunks, K split
]


@pytest.mark.parametrize("B,C,N,p,H,W", PATCH_W_SHAPES)
def test_x6_patch_wgrad_is_f32_class(B, C, N, p, H, W):
    """The patch-staged split-bf16 weight gradient (MD2_CONV_PATCH on md2_conv_wgrad:
    one fetch and split of three input rows per 32-pixel segment, nine shifted tiles)
    against fp64: f32-class like the per-tap x6 kernel and within 2e-6 of it;
    deterministic."""
    torch.manual_seed(41 + C + N + H + W)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL)
    w = (torch.randn(N, C, 3, 3, device="cuda") / (C * 9) ** 0.5).contiguous(memory_format=CL)
    gy = torch.randn(F.conv2d(x, w, None, 1, p).shape, device="cuda").contiguous(memory_format=CL)
    wref = torch.ops.aten.convolution_backward(gy.double().cpu(), x.double().cpu(), w.double().cpu(), None, (1, 1),
                                               (p, p), (1, 1), False, (0, 0), 1, (False, True, False))[1]
    w_mi = torch.ops.aten.convolution_backward(gy, x, w, None, (1, 1), (p, p), (1, 1), False, (0, 0), 1,
                                               (False, True, False))[1].double().cpu()
    e_mi = _rel(w_mi, wref)
    fl = conv_ops.X6 | conv_ops.PATCH
    gw = conv_ops._wgrad(gy, x, w, 1, p, fl)
    e = _rel(gw.double().cpu(), wref)
    assert e < max(3 * e_mi, 1e-7) and e < 2e-6, (e, e_mi)
    assert _rel(gw.double().cpu(), conv_ops._wgrad(gy, x, w, 1, p, conv_ops.X6).double().cpu()) < 2e-6
    assert torch.equal(gw, conv_ops._wgrad(gy, x, w, 1, p, fl))
