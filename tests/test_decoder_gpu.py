"""DepthDecoder block fusion (decoder_ops.conv_input, HIP) vs the eager
ELU / nearest-upsample / cat / ReflectionPad2d chain of the reference decoder
(networks/depth_decoder.py:50-65) on the same weights: outputs and gradients."""
import pytest
import torch

from monodepth2_amd import networks
from monodepth2_amd.decoder_ops import conv_input

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nhwc,C", [(False, 8), (True, 8), (True, 6)])   # NHWC C=8: float4 kernels, C=6: scalar
@pytest.mark.parametrize("elu,up,skip_ch", [(False, False, 0), (True, True, 0), (True, True, 64),
                                            (True, False, 0), (False, True, 32)])
def test_conv_input_matches_eager(elu, up, skip_ch, nhwc, C):
    torch.manual_seed(0)
    fmt = torch.channels_last if nhwc else torch.contiguous_format
    x = torch.randn(3, C, 6, 10, device="cuda").contiguous(memory_format=fmt).requires_grad_(True)
    H, W = (12, 20) if up else (6, 10)
    skip = (torch.randn(3, skip_ch, H, W, device="cuda").contiguous(memory_format=fmt).requires_grad_(True)
            if skip_ch else None)
    out = conv_input(x, skip, elu=elu, upsample=up, nhwc=nhwc)
    assert out.is_contiguous(memory_format=fmt)
    y = torch.nn.functional.elu(x) if elu else x
    if up:
        y = torch.nn.functional.interpolate(y, scale_factor=2, mode="nearest")
    if skip is not None:
        y = torch.cat([y, skip], 1)
    ref = torch.nn.functional.pad(y, (1, 1, 1, 1), mode="reflect")
    assert torch.equal(out, ref)
    g = torch.randn_like(ref)
    gx, = torch.autograd.grad(out, x, g.contiguous(memory_format=fmt), retain_graph=True)
    gxr, = torch.autograd.grad(ref, x, g, retain_graph=True)
    assert gx.is_contiguous(memory_format=fmt)
    torch.testing.assert_close(gx, gxr, rtol=1e-5, atol=1e-6)
    if skip is not None:
        gs, = torch.autograd.grad(out, skip, g, retain_graph=True)
        gsr, = torch.autograd.grad(ref, skip, g)
        torch.testing.assert_close(gs, gsr, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("C", [16, 32, 256])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("up,skip_ch", [(True, 64), (False, 0)])
def test_conv_input_folds_the_conv_bias(C, dtype, up, skip_ch):
    """conv_input(x, bias=b) == eager pad(cat(up(elu(x + b)), skip)); grads w.r.t. x, skip
    and b (the fused fixed-order bias-gradient reduction vs autograd's sum)."""
    torch.manual_seed(1)
    cl = torch.channels_last
    x = torch.randn(4, C, 12, 20, device="cuda").to(dtype).contiguous(memory_format=cl).requires_grad_(True)
    b = torch.randn(C, device="cuda", requires_grad=True)
    H, W = (24, 40) if up else (12, 20)
    skip = (torch.randn(4, skip_ch, H, W, device="cuda").to(dtype).contiguous(memory_format=cl).requires_grad_(True)
            if skip_ch else None)
    out = conv_input(x, skip, elu=True, upsample=up, nhwc=True, bias=b)
    y = torch.nn.functional.elu(x.float() + b.view(1, -1, 1, 1))
    if up:
        y = torch.nn.functional.interpolate(y, scale_factor=2, mode="nearest")
    if skip is not None:
        y = torch.cat([y, skip.float()], 1)
    ref = torch.nn.functional.pad(y, (1, 1, 1, 1), mode="reflect")
    tol = dict(rtol=1e-6, atol=1e-6) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(out.float(), ref, **tol)
    g = torch.randn(ref.shape, device="cuda")
    gx, gb = torch.autograd.grad(out, (x, b), g.to(dtype).contiguous(memory_format=cl), retain_graph=True)
    gxr, gbr = torch.autograd.grad(ref, (x, b), g.to(dtype).float())
    torch.testing.assert_close(gx.float(), gxr.float(), **tol)
    torch.testing.assert_close(gb, gbr, rtol=1e-4 if dtype == torch.float32 else 2e-2, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("up,skip_ch", [(False, 0), (True, 16)])
@pytest.mark.parametrize("used", [(0, 1), (0,), (1,)])
def test_conv_input_alias_sums_both_gradients(up, skip_ch, used, dtype):
    """conv_input(..., alias=True) -> (P, P'): the two consumers' gradients of the padded
    map are summed as the pad backward reads them (md2_decoder_pad_bwd2); grads w.r.t.
    x, skip and the folded bias match autograd's sum over the consumers."""
    torch.manual_seed(5)
    cl = torch.channels_last
    x = torch.randn(2, 32, 12, 20, device="cuda").to(dtype).contiguous(memory_format=cl).requires_grad_(True)
    b = torch.randn(32, device="cuda", requires_grad=True)
    H, W = (24, 40) if up else (12, 20)
    skip = (torch.randn(2, skip_ch, H, W, device="cuda").to(dtype).contiguous(memory_format=cl).requires_grad_(True)
            if skip_ch else None)
    P, P2 = conv_input(x, skip, elu=True, upsample=up, nhwc=True, bias=b, alias=True)
    assert torch.equal(P, P2) and "ConvInput" in type(P2.grad_fn).__name__
    gs = [torch.randn(P.shape, device="cuda").to(dtype).contiguous(memory_format=cl) for _ in range(2)]
    inputs = (x, b) + ((skip,) if skip is not None else ())
    got = torch.autograd.grad([(P, P2)[i] for i in used], inputs, [gs[i] for i in used])
    ref = conv_input(x, skip, elu=True, upsample=up, nhwc=True, bias=b)
    exp = torch.autograd.grad([ref] * len(used), inputs, [gs[i] for i in used])
    # bf16: autograd rounds the two consumers' sum to bf16 before the pad backward, the
    # fused path adds them in fp32 — one bf16 rounding apart
    t0, t1 = ((1e-6, 1e-6), (1e-5, 1e-4)) if dtype == torch.float32 else ((2e-2, 2e-2), (2e-2, 2e-2))
    torch.testing.assert_close(got[0].float(), exp[0].float(), rtol=t0[0], atol=t0[1])
    torch.testing.assert_close(got[1], exp[1], rtol=t1[0], atol=t1[1] * (1 if dtype == torch.float32 else 50))
    if skip is not None:
        torch.testing.assert_close(got[2].float(), exp[2].float(), rtol=t0[0], atol=t0[1])


def test_conv_input_bf16_matches_eager():
    """bf16 NHWC (--amp bf16): copies are exact, ELU rounded once to bf16."""
    torch.manual_seed(3)
    CL = torch.channels_last
    x = torch.randn(2, 16, 6, 10, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    skip = torch.randn(2, 32, 12, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    skip.requires_grad_(True)
    out = conv_input(x, skip, elu=True, upsample=True, nhwc=True)
    y = torch.cat([torch.nn.functional.interpolate(torch.nn.functional.elu(x.float()), scale_factor=2,
                                                   mode="nearest"), skip.float()], 1)
    ref = torch.nn.functional.pad(y, (1, 1, 1, 1), mode="reflect")
    assert out.dtype == torch.bfloat16 and out.is_contiguous(memory_format=CL)
    assert torch.equal(out.float(), ref.to(torch.bfloat16).float())
    g = torch.randn_like(ref).to(torch.bfloat16)
    gx, gs = torch.autograd.grad(out, (x, skip), g.contiguous(memory_format=CL))
    gxr, gsr = torch.autograd.grad(ref, (x, skip), g.float())
    torch.testing.assert_close(gx.float(), gxr.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(gs.float(), gsr.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("C,h,w", [(16, 96, 320), (32, 48, 160), (64, 24, 80), (128, 12, 40), (4, 5, 7),
                                   (256, 3, 9)])
@pytest.mark.parametrize("w_cl", [True, False])
def test_disp_head_matches_conv_sigmoid(C, h, w, w_cl):
    """decoder_ops.disp_head (md2_disp_head_*) vs sigmoid(Conv2d(C, 1, 3)) on MIOpen:
    disp and the gradients w.r.t. the padded input, weight and bias (fp32 tolerance:
    reduction order differs; the weight/bias sums run over B*h*w pixels)."""
    from monodepth2_amd.decoder_ops import disp_head
    torch.manual_seed(5)
    CL = torch.channels_last
    conv = torch.nn.Conv2d(C, 1, 3).cuda()
    if w_cl:
        conv = conv.to(memory_format=CL)
    P = torch.randn(3, C, h + 2, w + 2, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    d = disp_head(P, conv)
    ref = torch.sigmoid(conv(P))
    torch.testing.assert_close(d, ref, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(ref)
    gP, gw, gb = torch.autograd.grad(d, (P, conv.weight, conv.bias), g)
    gPr, gwr, gbr = torch.autograd.grad(ref, (P, conv.weight, conv.bias), g)
    assert gw.is_contiguous(memory_format=CL) == w_cl or C == 1
    torch.testing.assert_close(gP, gPr, rtol=1e-5, atol=1e-6)
    # weight/bias gradients are sums over B*h*w (up to 92k) products: measure both fp32
    # orders against fp64 and require ours no worse than 2x MIOpen's drift (+ a floor)
    P64, w64, b64 = P.detach().double().requires_grad_(True), conv.weight.detach().double(), conv.bias.detach().double()
    w64.requires_grad_(True)
    b64.requires_grad_(True)
    gw64, gb64 = torch.autograd.grad(torch.sigmoid(torch.nn.functional.conv2d(P64, w64, b64)), (w64, b64), g.double())
    for ours, theirs, exact in ((gw, gwr, gw64), (gb, gbr, gb64)):
        e_ours = (ours.double() - exact).abs().max().item()
        e_ref = (theirs.double() - exact).abs().max().item()
        assert e_ours <= 2 * e_ref + 2e-6 * exact.abs().max().item() + 1e-6, (e_ours, e_ref)


@pytest.mark.parametrize("C,h,w", [(16, 96, 320), (32, 48, 160), (64, 24, 80), (128, 12, 40), (4, 5, 7)])
@pytest.mark.parametrize("w_cl", [True, False])
def test_disp_head_bf16_input_is_the_fp32_head_on_its_values(C, h, w, w_cl):
    """MD2_HEAD_BF16 (ABI 23, config C5): the head reading a bf16 padded input equals the
    fp32 head on the same values widened, bit for bit (disp, weight and bias gradients),
    and its input gradient is that fp32 gradient rounded to bf16 (nearest even)."""
    from monodepth2_amd.decoder_ops import disp_head
    torch.manual_seed(6)
    CL = torch.channels_last
    conv = torch.nn.Conv2d(C, 1, 3).cuda()
    if w_cl:
        conv = conv.to(memory_format=CL)
    Pb = torch.randn(3, C, h + 2, w + 2, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    Pb.requires_grad_(True)
    Pf = Pb.detach().float().contiguous(memory_format=CL).requires_grad_(True)
    db_, df_ = disp_head(Pb, conv), disp_head(Pf, conv)
    assert db_.dtype == torch.float32 and torch.equal(db_, df_)
    g = torch.randn_like(df_)
    gPb, gwb, gbb = torch.autograd.grad(db_, (Pb, conv.weight, conv.bias), g)
    gPf, gwf, gbf = torch.autograd.grad(df_, (Pf, conv.weight, conv.bias), g)
    assert gPb.dtype == torch.bfloat16 and gPb.is_contiguous(memory_format=CL)
    assert torch.equal(gPb, gPf.to(torch.bfloat16))
    assert torch.equal(gwb, gwf) and torch.equal(gbb, gbf)


@pytest.mark.parametrize("num_layers,H,W,cl", [(18, 64, 128, False), (18, 192, 640, False), (50, 64, 96, False),
                                               (18, 64, 128, True)])
def test_fused_decoder_matches_eager(num_layers, H, W, cl):
    torch.manual_seed(0)
    enc = networks.ResnetEncoder(num_layers, False).cuda()
    dec = networks.DepthDecoder(enc.num_ch_enc, range(4)).cuda()
    if cl:   # channels_last build (--channels_last): NHWC convs and fused conv inputs
        enc, dec = enc.to(memory_format=torch.channels_last), dec.to(memory_format=torch.channels_last)
    img = torch.rand(2, 3, H, W, device="cuda")
    feats = [f.detach().requires_grad_(True) for f in enc(img)]
    dec.fused = True
    out_f = dec(feats)
    loss_f = sum((out_f[("disp", s)] * (s + 1)).sum() for s in range(4))
    g_f = torch.autograd.grad(loss_f, feats + list(dec.parameters()))
    dec.fused = False
    out_e = dec(feats)
    loss_e = sum((out_e[("disp", s)] * (s + 1)).sum() for s in range(4))
    g_e = torch.autograd.grad(loss_e, feats + list(dec.parameters()))
    for s in range(4):
        torch.testing.assert_close(out_f[("disp", s)], out_e[("disp", s)], rtol=1e-5, atol=1e-6)
    for a, b in zip(g_f, g_e):
        torch.testing.assert_close(a, b, rtol=2e-4, atol=1e-5)


@pytest.mark.parametrize("inv", [[True, False], [False, False, True]])
def test_fused_pose_matches_eager(inv):
    """pose_ops (HIP) vs layers.transformation_from_parameters (pinned by the golden
    axisangle/translation gradients) — values and gradients, incl. a zero rotation."""
    from monodepth2_amd.layers import transformation_from_parameters
    from monodepth2_amd.pose_ops import poses_to_transforms
    torch.manual_seed(1)
    F_, B = len(inv), 5
    aa = (0.1 * torch.randn(F_, B, 3, device="cuda")).requires_grad_(True)
    with torch.no_grad():
        aa[0, 0] = 0.0
    tr = torch.randn(F_, B, 3, device="cuda", requires_grad=True)
    T = poses_to_transforms(aa, tr, inv)
    Tr = torch.stack([transformation_from_parameters(aa[i].unsqueeze(1), tr[i].unsqueeze(1), invert=v)
                      for i, v in enumerate(inv)])
    torch.testing.assert_close(T, Tr, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(T)
    ga, gt = torch.autograd.grad(T, (aa, tr), g, retain_graph=True)
    gar, gtr = torch.autograd.grad(Tr, (aa, tr), g)
    torch.testing.assert_close(ga, gar, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gt, gtr, rtol=1e-5, atol=1e-6)


def test_packed_pose_producer_matches_split():
    """pose_ops.packed_poses_to_transforms on a strided (F,B,6) view of the pose
    decoder output == poses_to_transforms on its axisangle / translation halves,
    values and the gradient w.r.t. the packed tensor."""
    from monodepth2_amd.pose_ops import packed_poses_to_transforms, poses_to_transforms
    torch.manual_seed(2)
    F_, B = 2, 5
    raw = (0.1 * torch.randn(F_ * B, 2, 1, 6, device="cuda")).requires_grad_(True)   # (pairs*B, frames, 1, 6)
    x6 = raw[:, 0, 0].view(F_, B, 6)
    T = packed_poses_to_transforms(x6, [True, False])
    Tr = poses_to_transforms(x6[..., :3], x6[..., 3:], [True, False])
    assert torch.equal(T, Tr)
    g = torch.randn_like(T)
    gp, = torch.autograd.grad(T, raw, g)
    gr, = torch.autograd.grad(Tr, raw, g)
    assert torch.equal(gp, gr)


@pytest.mark.parametrize("cin,cout,k,relu", [(512, 256, 1, True), (256, 256, 3, True), (256, 12, 1, False)])
def test_conv_bias_act_matches_eager(cin, cout, k, relu):
    """decoder_ops.conv_bias_act (bias-free conv_ops convolution — split-bf16 MFMA or
    MIOpen, chosen per shape — + md2_bias_act_*) vs the pose decoder's eager
    relu(conv(x)): values and the gradients w.r.t. x, weight, bias (f32-class sums in
    different orders)."""
    from monodepth2_amd.decoder_ops import conv_bias_act
    torch.manual_seed(4)
    CL = torch.channels_last
    conv = torch.nn.Conv2d(cin, cout, k, 1, k // 2).cuda().to(memory_format=CL)
    x = torch.randn(6, cin, 6, 20, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    y = conv_bias_act(conv, x, relu)
    assert y.grad_fn is not None and "BiasAct" in type(y.grad_fn).__name__
    ref = conv(x)
    ref = torch.relu(ref) if relu else ref
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    g = torch.randn_like(ref)
    got = torch.autograd.grad(y, (x, conv.weight, conv.bias), g)
    exp = torch.autograd.grad(ref, (x, conv.weight, conv.bias), g)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("relu,C", [(True, 256), (False, 12)])
def test_bf16_bias_act_matches_autocast(relu, C):
    """decoder_ops._BiasActBF16 (C5's pose decoder bias + ReLU): the forward bitwise
    autocast's bf16 add + ReLU, the input gradient bitwise torch's threshold_backward, the
    bias gradient within one bf16 ulp of the fp64 sum of the same bf16 gradient; bitwise
    repeatable."""
    from monodepth2_amd.decoder_ops import _BiasActBF16
    torch.manual_seed(C)
    z = torch.randn(4, C, 6, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(C, device="cuda")
    g = torch.randn(z.shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def ours():
        zz, bb = z.clone().requires_grad_(True), b.clone().requires_grad_(True)
        y = _BiasActBF16.apply(zz, bb, relu)
        gz, gb = torch.autograd.grad(y, [zz, bb], g)
        return y, gz, gb

    zz, bb = z.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = zz + bb.to(torch.bfloat16).view(1, -1, 1, 1)
    yr = torch.relu(yr) if relu else yr
    gzr, gbr = torch.autograd.grad(yr, [zz, bb], g)
    y, gz, gb = ours()
    assert torch.equal(y, yr) and torch.equal(gz, gzr)
    ref = (g.double() * (yr.double() > 0) if relu else g.double()).sum((0, 2, 3))
    assert bool(((gb.double() - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-6).all())
    assert torch.equal(gb, gb.to(torch.bfloat16).float())
    y2, gz2, gb2 = ours()
    assert torch.equal(gb, gb2) and torch.equal(gz, gz2)
