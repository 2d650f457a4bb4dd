"""GPU parity: the HIP hot path (through the C ABI) against the reference's golden
vectors (tests/golden/*.npz, captured from /root/reference by make_golden.py) and
against the oracle on the same seeded inputs.

Two tiers (fp32; north_star asks loss delta < 1e-4):

1. against the reference's golden vectors:
   * losses: |delta| <= 2e-6 per scale and total;
   * warped colours / samples / depth: abs 2e-5 / 2e-5 / rel 1e-5;
   * per-pixel argmin (identity_selection): at most max(2, 1e-4 * pixels) flips
     per scale.  A flip happens only where two candidates tie to within fp32
     rounding (gaps of 3e-8..6e-7 observed, tools/parity_report.py) and it
     re-routes that pixel's gradient, so:
   * gradients: relative L2 error <= 2e-2 per tensor.
2. against the oracle on the same inputs with the argmin PINNED to the HIP
   selection (oracle `selection=`), which isolates the gradient math from the
   tie flips: losses <= 2e-6; >= 99 % of gradient pixels within
   1e-4*max|ref| + 1e-3*|ref| and relative L2 <= 1e-2.  The remaining pixels are
   where a sample coordinate lies within fp32 rounding of an integer (the bilinear
   derivative is discontinuous there, so the two implementations pick different
   cells) or where SSIM's clamp at 0 ties; measured: 0-10 pixels per tensor,
   typical relative L2 1e-5 (small cases) to 4e-3 (the coarsest scale at
   640x192, where one pixel aggregates 256 full-resolution gradients).
   Sample-grid coordinates of near-singular projections (points behind or at the
   camera plane, |value| up to 3e5) are compared at 1e-2 relative beyond |100|.

At full size (640x192, 1024x320, mono+stereo) more samples land within rounding of
a cell boundary and the coarse-scale gradients aggregate them, so the fixed bars
are widened to what the reference's OWN formulation drifts on a second fp32
platform: the same ATen ops run on PyTorch-ROCm (`run_oracle(device="cuda")`,
a yardstick only) against the CPU goldens / CPU oracle.  The HIP path must stay
within 3x that drift (relative L2) and 0.5 % of it (fraction of pixels in
tolerance); against the goldens (argmin not pinned) the disparity pixels whose
gradient footprint touches an argmin flip are left out (flip_footprint), the flips
themselves bounded as above.  Measured (tools/parity_platforms.py), pinned:
stereo 640x192 scale 2 rel-L2 HIP 1.4e-2 vs ATen-GPU 2.0e-2, scale 3 1.2e-2 vs
6.0e-3; 1024x320 scale 3 in-tolerance HIP 98.6 % vs ATen-GPU 98.8 %.  Argmin flips
per scale vs the CPU reference: HIP 4-58, ATen-GPU 2-43 (out of 245,760-655,360
pixels).
"""
import numpy as np
import pytest
import torch

from golden_io import Case, case_names
from hotpath_case import run_hip, run_oracle

pytestmark = pytest.mark.gpu


def flip_footprint(flips, s):
    """Disparity pixels at scale s (B,1,h,w) whose gradient reads a full-resolution
    pixel within one pixel of an argmin flip (SSIM's 3x3 adjoint, then the bilinear
    upsample's 2x2 source footprint, align_corners=False)."""
    f = torch.from_numpy(flips.astype(np.float32)).unsqueeze(1)
    dil = torch.nn.functional.max_pool2d(f, 3, 1, 1)[:, 0].numpy() > 0
    B, H, W = dil.shape
    h, w = H >> s, W >> s
    y0 = np.minimum(np.floor(np.maximum((np.arange(H) + 0.5) / 2 ** s - 0.5, 0)).astype(int), h - 1)
    x0 = np.minimum(np.floor(np.maximum((np.arange(W) + 0.5) / 2 ** s - 0.5, 0)).astype(int), w - 1)
    y1, x1 = np.minimum(y0 + 1, h - 1), np.minimum(x0 + 1, w - 1)
    mask = np.zeros((B, 1, h, w), bool)
    b, yy, xx = np.nonzero(dil)
    for ys in (y0, y1):
        for xs in (x0, x1):
            mask[b, 0, ys[yy], xs[xx]] = True
    return mask


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", case_names())
def test_hip_matches_reference(name):
    case = Case(name)
    cfg, out = run_hip(case)
    for s in range(4):
        assert abs(out["loss"][s] - float(case.expected(f"loss_{s}"))) <= 2e-6, (s, out["loss"][s])
    assert abs(out["loss"][4] - float(case.expected("loss"))) <= 2e-6
    if case.full:
        for s in range(4):
            for fi, f in enumerate(case.frame_ids[1:]):
                np.testing.assert_allclose(out["gen"]["color"][(fi, s)].cpu().numpy(),
                                           case.expected(f"warp_{f}_{s}"), atol=2e-5)
                got, want = out["gen"]["sample"][(fi, s)].cpu().numpy(), case.expected(f"sample_{f}_{s}")
                near = np.abs(want) < 100.0   # far out-of-frame points are clamped to the border anyway
                np.testing.assert_allclose(got[near], want[near], atol=2e-5, rtol=1e-3)
                np.testing.assert_allclose(got[~near], want[~near], rtol=1e-2)
            np.testing.assert_allclose(out["gen"]["depth"][s].cpu().numpy(), case.expected(f"depth_{s}"),
                                       rtol=1e-5)
            if "disable_automasking" not in case.flags:
                C = 1 if cfg.avg_reprojection else cfg.num_src
                ident_sel = (out["select"][s] > C - 1).astype(np.uint8)
                flips = int((ident_sel != case.expected(f"identity_selection_{s}")).sum())
                assert flips <= max(2, 1e-4 * ident_sel.size), (s, flips)
    else:
        for s in range(4):
            if "disable_automasking" not in case.flags:
                C = 1 if cfg.avg_reprojection else cfg.num_src
                m = float((out["select"][s] > C - 1).mean())
                assert abs(m - float(case.expected(f"identity_selection_mean_{s}"))) < 1e-3
    if case.full is False and "disable_automasking" not in case.flags:
        # full size: compare away from the argmin flips (each re-routes a pixel's
        # gradient to another candidate); the flips themselves are bounded above
        cpu = run_oracle(case)
        aten = run_oracle(case, device="cuda")
        C = 1 if cfg.avg_reprojection else cfg.num_src
        for s in range(4):
            ref_sel = cpu["outputs"][f"identity_selection/{s}"].cpu().numpy() > 0.5
            ident_flips = (out["select"][s] > C - 1) != ref_sel
            assert ident_flips.sum() <= max(2, 1e-4 * ident_flips.size), (s, int(ident_flips.sum()))
            # any argmin difference (also between two reprojection candidates)
            flips = out["select"][s] != cpu["outputs"][f"argmin/{s}"].cpu().numpy()
            keep = ~flip_footprint(flips, s)
            want = case.expected(f"grad_disp_{s}")
            e = rel_l2(out["grad_disp"][s][keep], want[keep])
            # the reference's own drift on this machine: the same ATen ops on the GPU,
            # and on this host's CPU (its vector kernels need not sum in the order of
            # the machine that wrote the goldens)
            drift = max(rel_l2(aten["grad_disp"][s][keep], want[keep]),
                        rel_l2(cpu["grad_disp"][s][keep], want[keep]))
            bar = max(2e-2, 3 * drift)
            assert e <= bar, (s, e, bar)
    else:
        for s in range(4):
            e = rel_l2(out["grad_disp"][s], case.expected(f"grad_disp_{s}"))
            assert e <= 2e-2, (s, e)
    assert rel_l2(out["grad_axis"], case.expected("grad_axisangle")) <= 2e-2
    assert rel_l2(out["grad_trans"], case.expected("grad_translation")) <= 2e-2
    for i, f in enumerate(case.temporal):
        assert rel_l2(out["grad_T"][case.frame_ids[1:].index(f)], case.expected(f"grad_T_{f}")) <= 2e-2
    for s, g in out.get("grad_mask", {}).items():
        assert rel_l2(g, case.expected(f"grad_mask_{s}")) <= 2e-2, (s, rel_l2(g, case.expected(f"grad_mask_{s}")))


@pytest.mark.parametrize("name", case_names())
def test_hip_gradients_match_oracle_pinned_selection(name):
    case = Case(name)
    cfg, out = run_hip(case)
    sel = None if cfg.disable_automasking and cfg.avg_reprojection else out["select"]
    ref = run_oracle(case, selection=sel)
    aten = run_oracle(case, selection=sel, device="cuda") if case.full is False else None
    for s in range(5):
        assert abs(out["loss"][s] - ref["loss"][s]) <= 2e-6, (s, out["loss"][s], ref["loss"][s])

    def in_tol(g, r):
        return float((np.abs(g - r) <= 1e-4 * np.abs(r).max() + 1e-3 * np.abs(r)).mean())

    for s in range(4):
        g, r = out["grad_disp"][s], ref["grad_disp"][s]
        frac_bar, rel_bar = 0.99, 1e-2
        if aten is not None:
            a = aten["grad_disp"][s]
            frac_bar = min(frac_bar, in_tol(a, r) - 0.005)
            rel_bar = max(rel_bar, 3 * rel_l2(a, r))
        assert in_tol(g, r) >= frac_bar, (s, in_tol(g, r), frac_bar)
        assert rel_l2(g, r) <= rel_bar, (s, rel_l2(g, r), rel_bar)
    assert rel_l2(out["grad_axis"], ref["grad_axis"]) <= 1e-2
    assert rel_l2(out["grad_trans"], ref["grad_trans"]) <= 1e-2
    for s, g in out.get("grad_mask", {}).items():
        assert rel_l2(g, ref["grad_mask"][s]) <= 1e-2, s


def test_hip_deterministic():
    case = Case("mono_b2_64x128")
    _, a = run_hip(case)
    _, b = run_hip(case)
    assert np.array_equal(a["loss"], b["loss"])
    for s in range(4):
        assert np.array_equal(a["grad_disp"][s], b["grad_disp"][s])
    assert np.array_equal(a["grad_T"], b["grad_T"])


@pytest.mark.parametrize("name", ["mono_b2_64x128", "stereo_b2_64x128"])
def test_seeded_noise_path_matches_oracle(name):
    """The production path draws the tie-break noise in-kernel (noise=None, seed).
    md2_tiebreak_noise exports that exact draw; handed to the oracle it must give
    the same losses (<= 2e-6) and argmin maps (flips only at fp32 near-ties), and
    the draw itself must look unit normal (trainer.py:468 uses torch.randn)."""
    from monodepth2_amd.hotpath import tiebreak_noise
    case = Case(name)
    case.noise = None
    cfg, out_a = run_hip(case)                    # seed 0
    noise = tiebreak_noise(cfg, seed=0)
    for s in range(4):
        n = noise[s].double()
        assert abs(float(n.mean())) < 0.03 and abs(float(n.std()) - 1.0) < 0.03, (s, float(n.mean()), float(n.std()))
        if s > 0:
            assert not torch.equal(noise[s], noise[0])   # fresh draw per scale
    case.noise = {s: n.cpu() for s, n in noise.items()}
    ref = run_oracle(case)
    for s in range(5):
        assert abs(out_a["loss"][s] - ref["loss"][s]) <= 2e-6, (s, out_a["loss"][s], ref["loss"][s])
    C = cfg.num_src
    for s in range(4):
        flips = int(((out_a["select"][s] > C - 1) != (ref["outputs"][f"identity_selection/{s}"].cpu().numpy() > 0.5)).sum())
        assert flips <= max(2, 1e-4 * out_a["select"][s].size), (s, flips)
    # an explicit noise tensor equal to the in-kernel draw selects identically
    _, out_b = run_hip(case)
    for s in range(4):
        assert np.array_equal(out_a["select"][s], out_b["select"][s])


@pytest.mark.parametrize("name", ["mono_b2_64x128", "stereo_b2_64x128", "mono_bigpose_b2_64x96"])
def test_eight_bit_sources_match_oracle(name):
    """Colours that are exactly k/255 (the loader's to_tensor output,
    datasets/mono_dataset.py:199-200) take the 8-bit RGBx gather path
    (pack_src8_kernel); against the oracle on the same quantised inputs, argmin
    pinned to the HIP selection, the bars of the fp32 path hold."""
    case = Case(name)
    for k, v in list(case.inputs.items()):
        if isinstance(k, tuple) and k[0] in ("color", "color_aug"):
            case.inputs[k] = torch.round(v * 255.0) / 255.0
    cfg, out = run_hip(case)
    ref = run_oracle(case, selection=out["select"])
    for s in range(5):
        assert abs(out["loss"][s] - ref["loss"][s]) <= 2e-6, (s, out["loss"][s], ref["loss"][s])
    for s in range(4):
        g, r = out["grad_disp"][s], ref["grad_disp"][s]
        assert float((np.abs(g - r) <= 1e-4 * np.abs(r).max() + 1e-3 * np.abs(r)).mean()) >= 0.99, s
        assert rel_l2(g, r) <= 1e-2, (s, rel_l2(g, r))
    assert rel_l2(out["grad_axis"], ref["grad_axis"]) <= 1e-2
    assert rel_l2(out["grad_trans"], ref["grad_trans"]) <= 1e-2
    # the warped colours the 8-bit gathers produce (generate_images reads fp32) agree
    # through the loss: an unpinned run selects the same candidates up to near-ties
    ref_free = run_oracle(case)
    C = cfg.num_src
    for s in range(4):
        flips = int(((out["select"][s] > C - 1)
                     != (ref_free["outputs"][f"identity_selection/{s}"].cpu().numpy() > 0.5)).sum())
        assert flips <= max(2, 1e-4 * out["select"][s].size), (s, flips)
