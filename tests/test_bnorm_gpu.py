"""Fused NHWC BatchNorm2d (+ residual) (+ ReLU) (csrc/bnorm.hip via bn_ops.bn_act) vs
nn.BatchNorm2d + add + ReLU on the same module: outputs, running statistics and
gradients (x, weight, bias, residual), at every ResNet-18/50 width."""
import copy

import pytest
import torch
import torch.nn as nn

from monodepth2_amd import bn_ops, networks

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _eager(bn, x, r, relu):
    y = bn(x)
    if r is not None:
        y = y + r
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("C,shape", [(64, (3, 48, 160)), (128, (2, 24, 80)), (256, (2, 12, 40)),
                                     (512, (12, 6, 20)), (2048, (2, 3, 5)), (64, (1, 1, 2)),
                                     (1024, (2, 4, 8)), (2048, (2, 2, 4)), (256, (2, 16, 32)), (512, (2, 8, 16))])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_act_matches_batchnorm(C, shape, relu, res):
    torch.manual_seed(0)
    B, H, W = shape
    bn = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.9, 1.1)
    ref_bn = copy.deepcopy(bn)
    x = (torch.randn(B, C, H, W, device="cuda") * 2 + 0.7).contiguous(memory_format=CL).requires_grad_(True)
    r = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=CL).requires_grad_(True) if res else None
    xr = x.detach().clone().requires_grad_(True)
    rr = r.detach().clone().requires_grad_(True) if res else None
    y = bn_ops.bn_act(bn, x, r, relu)
    yr = _eager(ref_bn, xr, rr, relu)
    assert y.is_contiguous(memory_format=CL)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1
    g = torch.randn_like(yr)
    ins = [x, bn.weight, bn.bias] + ([r] if res else [])
    ins_r = [xr, ref_bn.weight, ref_bn.bias] + ([rr] if res else [])
    got = torch.autograd.grad(y, ins, g.contiguous(memory_format=CL))
    ref = torch.autograd.grad(yr, ins_r, g)
    for a, b, name in zip(got, ref, ["x", "weight", "bias", "residual"]):
        scale = float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= 2e-4 * scale + 1e-6, name


@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_act_bf16_matches_batchnorm_fp32(relu, res):
    """bf16 storage (--amp bf16): vs nn.BatchNorm2d in fp32 on the same bf16 values,
    within bf16 rounding of the outputs / gradients."""
    torch.manual_seed(2)
    C, B, H, W = 128, 2, 24, 80
    bn = nn.BatchNorm2d(C).cuda()
    ref_bn = copy.deepcopy(bn)
    xb = (torch.randn(B, C, H, W, device="cuda") * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    rb = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL) if res else None
    x = xb.clone().requires_grad_(True)
    r = rb.clone().requires_grad_(True) if res else None
    xr = xb.float().requires_grad_(True)
    rr = rb.float().requires_grad_(True) if res else None
    y = bn_ops.bn_act(bn, x, r, relu)
    yr = _eager(ref_bn, xr, rr, relu)
    assert y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-4, atol=1e-5)
    g = torch.randn_like(yr)
    got = torch.autograd.grad(y, [x, bn.weight, bn.bias], g.to(torch.bfloat16).contiguous(memory_format=CL))
    ref = torch.autograd.grad(yr, [xr, ref_bn.weight, ref_bn.bias], g.to(torch.bfloat16).float())
    for a, b in zip(got, ref):
        assert float((a.float() - b).norm() / b.norm()) < 1e-2


@pytest.mark.parametrize("bf16", [False, True])
def test_bn_groups_equal_separate_calls(bf16):
    """bn_groups(2) over a 2-chunk batch == two BatchNorm calls (per-chunk statistics,
    running statistics updated chunk after chunk)."""
    torch.manual_seed(4)
    C, B, H, W = 64, 6, 12, 20
    dt = torch.bfloat16 if bf16 else torch.float32
    bn = nn.BatchNorm2d(C).cuda()
    ref_bn = copy.deepcopy(bn)
    xb = torch.randn(B, C, H, W, device="cuda")
    xb[B // 2:] = xb[B // 2:] * 3 - 1   # the chunks differ in statistics
    xb = xb.to(dt).contiguous(memory_format=CL)
    rb = torch.randn(B, C, H, W, device="cuda").to(dt).contiguous(memory_format=CL)
    x, r = xb.clone().requires_grad_(True), rb.clone().requires_grad_(True)
    xr, rr = xb.float().requires_grad_(True), rb.float().requires_grad_(True)
    with bn_ops.bn_groups(2):
        y = bn_ops.bn_act(bn, x, r)
    yr = torch.cat([_eager(ref_bn, xc, rc, True) for xc, rc in zip(xr.chunk(2), rr.chunk(2))], 0)
    tol = 1e-2 if bf16 else 2e-5
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 2
    g = torch.randn_like(yr)
    got = torch.autograd.grad(y, [x, r, bn.weight, bn.bias], g.to(dt).contiguous(memory_format=CL))
    ref = torch.autograd.grad(yr, [xr, rr, ref_bn.weight, ref_bn.bias], g.to(dt).float())
    for a, b in zip(got, ref):
        assert float((a.float() - b).norm() / b.norm()) < (1e-2 if bf16 else 1e-4)


def test_bn_act_deterministic():
    torch.manual_seed(1)
    bn = nn.BatchNorm2d(64).cuda()
    x = torch.randn(12, 64, 96, 320, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    outs = []
    for _ in range(2):
        y = bn_ops.bn_act(bn, x)
        gx, gw = torch.autograd.grad(y, [x, bn.weight], torch.ones_like(y))
        outs.append((y, gx, gw))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _grads(enc, img, fused):
    bn_ops.ENABLED = fused
    try:
        feats = enc(img)
    finally:
        bn_ops.ENABLED = True
    loss = sum((f * (i + 1)).mean() for i, f in enumerate(feats))
    return feats, torch.autograd.grad(loss, list(enc.parameters()), allow_unused=True)   # fc head unused


def _worst(ga, gb):
    return max(float((a - b).norm() / (b.norm() + 1e-12)) for a, b in zip(ga, gb) if b is not None)


@pytest.mark.parametrize("num_layers", [18, 50])
def test_encoder_fused_bn_matches_unfused(num_layers):
    """Whole ResNet encoder, channels_last, training mode: fused vs nn.BatchNorm2d.
    Deep layers normalise over few pixels at this size, which makes the encoder's
    gradient sensitive to rounding: the bar is the change a 1e-6 relative input
    perturbation causes in the unfused encoder itself (measured: R18 7e-5, R50 6-8 %;
    fused vs unfused R18 2.5e-5, R50 2-5 %)."""
    torch.manual_seed(0)
    enc = networks.ResnetEncoder(num_layers, False).cuda().to(memory_format=CL)
    ref, pert = copy.deepcopy(enc), copy.deepcopy(enc)
    img = torch.rand(2, 3, 64, 128, device="cuda")
    feats, gs = _grads(enc, img, True)
    feats_r, gr = _grads(ref, img, False)
    _, gp = _grads(pert, img * (1 + 1e-6 * torch.randn_like(img)), False)
    for a, b in zip(feats, feats_r):
        assert float((a - b).norm() / b.norm()) < 1e-4
    assert _worst(gs, gr) <= max(1e-3, _worst(gp, gr)), (_worst(gs, gr), _worst(gp, gr))
    for (n, a), (_, b) in zip(enc.named_buffers(), ref.named_buffers()):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.parametrize("shape,dt", [((2, 64, 96, 320), torch.float32), ((3, 64, 7, 9), torch.float32),
                                      ((2, 64, 24, 80), torch.bfloat16), ((1, 8, 1, 1), torch.float32)])
def test_maxpool_matches_aten(shape, dt):
    """MaxPool2d(3, 2, 1) on channels_last (csrc/pool.hip) vs ATen: values exact,
    gradients exact up to the sum order of overlapping windows; ties (ReLU zeros)
    resolved to the same element."""
    torch.manual_seed(5)
    pool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
    x0 = torch.relu(torch.randn(*shape, device="cuda")).to(dt).contiguous(memory_format=CL)   # many ties at 0
    x = x0.clone().requires_grad_(True)
    xr = x0.clone().requires_grad_(True)
    y = bn_ops.max_pool_3x3s2(pool, x)
    yr = pool(xr)
    assert y.is_contiguous(memory_format=CL)
    assert torch.equal(y, yr)
    g = torch.randn_like(yr)
    gx, = torch.autograd.grad(y, x, g.contiguous(memory_format=CL))
    gxr, = torch.autograd.grad(yr, xr, g)
    torch.testing.assert_close(gx.float(), gxr.float(), rtol=1e-5, atol=1e-6 if dt == torch.float32 else 2e-2)


def test_maxpool_nan_propagates():
    pool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
    x = torch.zeros(1, 4, 6, 6, device="cuda").contiguous(memory_format=CL)
    x[0, 1, 2, 3] = float("nan")
    y = bn_ops.max_pool_3x3s2(pool, x)
    assert torch.equal(torch.isnan(y), torch.isnan(pool(x)))


def test_maxpool_with_alias_sums_both_gradients():
    """max_pool_3x3s2_with_alias: the alias's gradient (the decoder skip of the stem
    activation) is added in the pool's backward gather (md2_maxpool3s2_bwd_add) —
    same gradient as autograd's sum over the two consumers."""
    torch.manual_seed(9)
    CL = torch.channels_last
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(2, 64, 24, 40, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    y, xa = bn_ops.max_pool_3x3s2_with_alias(pool, x)
    assert "MaxPool" in type(xa.grad_fn).__name__ and torch.equal(xa, x)
    gy, ga = torch.randn_like(y), torch.randn_like(x)
    gx, = torch.autograd.grad([y, xa], x, [gy, ga])
    yr = pool(x)
    gxr, = torch.autograd.grad([yr, x * 1.0], x, [gy, ga])
    torch.testing.assert_close(gx, gxr, rtol=1e-6, atol=1e-6)
    # alias unused: the plain pool adjoint
    y2, _ = bn_ops.max_pool_3x3s2_with_alias(pool, x)
    g2, = torch.autograd.grad(y2, x, gy)
    g2r, = torch.autograd.grad(pool(x), x, gy)
    torch.testing.assert_close(g2, g2r, rtol=1e-6, atol=1e-6)


def test_maxpool_alias_only_gradient():
    """Only the alias output reaches the loss (the pool output's gradient is None
    under set_materialize_grads(False)): the input gradient is the alias's."""
    torch.manual_seed(10)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(2, 64, 12, 20, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    _, xa = bn_ops.max_pool_3x3s2_with_alias(pool, x)
    ga = torch.randn_like(x)
    gx, = torch.autograd.grad(xa, x, ga)
    torch.testing.assert_close(gx, ga, rtol=0, atol=0)


@pytest.mark.parametrize("used", [(0, 1, 2), (0, 1), (1, 2), (0, 2), (1,), (2,)])
def test_maxpool_out_alias_sums_all_gradients(used):
    """out_alias: (y, y', x') — the pooled map's second consumer (the first block's
    shortcut) and the input's (the decoder skip) are summed in the pool's gather
    (md2_maxpool3s2_bwd_multi), for every subset of the three outputs that reaches
    the loss; same gradient as autograd's sum over the consumers."""
    torch.manual_seed(11)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(2, 64, 24, 40, device="cuda").contiguous(memory_format=CL).requires_grad_(True)
    outs = bn_ops.max_pool_3x3s2_with_alias(pool, x, out_alias=True)
    assert len(outs) == 3 and torch.equal(outs[1], outs[0]) and torch.equal(outs[2], x)
    grads = [torch.randn_like(o) for o in outs]
    gx, = torch.autograd.grad([outs[i] for i in used], x, [grads[i] for i in used])
    yr = pool(x)
    refs = [yr, yr * 1.0, x * 1.0]
    gxr, = torch.autograd.grad([refs[i] for i in used], x, [grads[i] for i in used])
    torch.testing.assert_close(gx, gxr, rtol=1e-6, atol=1e-6)


def test_maxpool_out_alias_bf16():
    torch.manual_seed(12)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(2, 64, 12, 20, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=CL)
    x.requires_grad_(True)
    y, y2, xa = bn_ops.max_pool_3x3s2_with_alias(pool, x, out_alias=True)
    gy, gy2, ga = torch.randn_like(y), torch.randn_like(y), torch.randn_like(x)
    gx, = torch.autograd.grad([y, y2, xa], x, [gy, gy2, ga])
    gxr, = torch.autograd.grad([pool(x.float())], x, [(gy.float() + gy2.float())])
    torch.testing.assert_close(gx.float(), (gxr.float() + ga.float()), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("groups", [1, 2])
@pytest.mark.parametrize("used", [(0, 1, 2), (0, 2), (1, 2)])
def test_bn_bwd_multi_sums_alias_gradients(bf16, groups, used):
    """bn_act(..., aliases=2): y and its two alias views get three different
    gradients; the fused backward (md2_bn_bwd_multi) sums them on load.  Reference:
    nn.BatchNorm2d (+ residual + ReLU) fed the sum of the gradients that reach it.
    `used` = which of (y, alias1, alias2) reach the loss (the others bring None)."""
    torch.manual_seed(11 + groups)
    C, B, H, W = 64, 4, 12, 20
    dt = torch.bfloat16 if bf16 else torch.float32
    bn = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    ref_bn = copy.deepcopy(bn)
    xb = (torch.randn(B, C, H, W, device="cuda") * 2 + 0.3).to(dt).contiguous(memory_format=CL)
    rb = torch.randn(B, C, H, W, device="cuda").to(dt).contiguous(memory_format=CL)
    x, r = xb.clone().requires_grad_(True), rb.clone().requires_grad_(True)
    xr, rr = xb.float().requires_grad_(True), rb.float().requires_grad_(True)
    with bn_ops.bn_groups(groups):
        outs = bn_ops.bn_act(bn, x, r, True, aliases=2)
    assert len(outs) == 3 and "BNAct" in type(outs[1].grad_fn).__name__
    yr = torch.cat([_eager(ref_bn, xc, rc, True) for xc, rc in zip(xr.chunk(groups), rr.chunk(groups))], 0)
    gs = [torch.randn_like(yr) * (k + 1) for k in range(3)]
    gs = [g.to(dt).float() for g in gs]
    got = torch.autograd.grad([outs[k] for k in used], [x, r, bn.weight, bn.bias],
                              [gs[k].to(dt).contiguous(memory_format=CL) for k in used])
    ref = torch.autograd.grad(yr, [xr, rr, ref_bn.weight, ref_bn.bias], sum(gs[k] for k in used))
    tol = 1e-2 if bf16 else 1e-4
    for a, b, name in zip(got, ref, ["x", "residual", "weight", "bias"]):
        assert float((a.float() - b).norm() / b.norm()) < tol, name


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("res,groups", [(False, 1), (True, 1), (False, 2)])
def test_relu_mask_path_is_bit_equal_to_y_path(dtype, res, groups):
    """ABI 15: md2_bn_fwd_mask writes y (bit-equal to md2_bn_fwd) plus one mask byte per
    element quad with bit i = (y[4q+i] > 0); md2_bn_bwd_mask gated by it gives the same
    bits as md2_bn_bwd_multi reading y.  x is offset so some bf16 outputs sit near 0."""
    import ctypes
    from monodepth2_amd import _lib
    torch.manual_seed(7)
    B, C, H, W = 4, 64, 12, 20
    x = (torch.randn(B, C, H, W, device="cuda") * 0.5).to(dtype).contiguous(memory_format=CL)
    r = torch.randn(B, C, H, W, device="cuda").to(dtype).contiguous(memory_format=CL) if res else None
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.rand(C, device="cuda") - 0.5
    flags = _lib.BN_RELU | (_lib.BN_RESIDUAL if res else 0) | (_lib.BN_BF16 if dtype == torch.bfloat16 else 0)
    d = _lib.BnDesc(B * H * W, C, flags, 1e-5, 0.1, groups, 0)
    L = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(L.md2_bn_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device="cuda")
    rp = r.data_ptr() if res else None
    outs = []
    for use_mask in (False, True):
        y = torch.empty_like(x)
        mean = torch.empty(groups, C, device="cuda")
        inv = torch.empty(groups, C, device="cuda")
        mask = torch.empty(x.numel() // 4, dtype=torch.uint8, device="cuda")
        if use_mask:
            _lib.check(L.md2_bn_fwd_mask(ctypes.byref(d), x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rp, None,
                                         None, y.data_ptr(), mask.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                         ws.data_ptr(), st), "fwd_mask")
        else:
            _lib.check(L.md2_bn_fwd(ctypes.byref(d), x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rp, None, None,
                                    y.data_ptr(), mean.data_ptr(), inv.data_ptr(), ws.data_ptr(), st), "fwd")
        g = torch.randn(B, C, H, W, device="cuda", generator=torch.Generator("cuda").manual_seed(3)).to(dtype)
        g = g.contiguous(memory_format=CL)
        gx, gr = torch.empty_like(x), (torch.empty_like(x) if res else None)
        gw, gb = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        args = (g.data_ptr(), None, None, gamma.data_ptr(), mean.data_ptr(), inv.data_ptr(), gx.data_ptr(),
                gr.data_ptr() if res else None, gw.data_ptr(), gb.data_ptr(), ws.data_ptr(), st)
        if use_mask:
            _lib.check(L.md2_bn_bwd_mask(ctypes.byref(d), x.data_ptr(), mask.data_ptr(), *args), "bwd_mask")
            # NHWC element e = 4 q + i: bit i of byte q
            bits = (mask.view(-1, 1).to(torch.int32) >> torch.arange(4, device="cuda")) & 1
            pos = (y.permute(0, 2, 3, 1).reshape(-1, 4).float() > 0).to(torch.int32)
            assert torch.equal(bits, pos)
        else:
            _lib.check(L.md2_bn_bwd_multi(ctypes.byref(d), x.data_ptr(), y.data_ptr(), *args), "bwd")
        outs.append([t for t in (y, mean, inv, gx, gr, gw, gb) if t is not None])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
