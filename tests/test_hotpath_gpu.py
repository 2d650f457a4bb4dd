"""GPU parity: the HIP hot path (through the C ABI) against the reference's golden
vectors (tests/golden/*.npz, captured from /root/reference by make_golden.py, which
also records the reference's own per-pixel argmin of trainer.py:478) and against the
oracle on the same inputs.  fp32 throughout; north_star asks loss delta < 1e-4.

Bars are fixed numbers, never recomputed at run time; the full-size gradient bars are
anchored on the reference formulation's own fp32 floor (profiles/r04/parity_floor.json,
tests/test_parity_floor_gpu.py), the rest set per case at about 3x what
tools/parity_measure.py measured on MI355X (profiles/r03/parity_measured.json):

* losses: |delta| <= 2e-6 per scale and total (measured <= 9.5e-7);
* warped colours / samples / depth (small cases): abs 2e-5 / 2e-5 / rel 1e-5;
* argmin flips (HIP selection vs the reference's argmin): at most max(3, 4e-4 *
  pixels) per scale (measured <= 1.3e-4).  A flip happens only where two candidates tie to within fp32
  rounding (gaps of 3e-8..6e-7, tools/parity_report.py) and re-routes that pixel's
  gradient, so gradients are compared outside its footprint (`flip_footprint`);
* tier 1 (vs the goldens, outside the flip footprint), small cases: relative L2 of
  dL/ddisp_s <= 1e-4 (measured 2e-6 .. 2.2e-5);
* tier 2 (vs the oracle with the argmin PINNED to the HIP selection): relative L2
  <= 1e-4 (measured <= 2e-5) on the small cases;
* full size (640x192 B=2 and B=12, 1024x320, mono+stereo): a handful of pixels per
  image have a sample coordinate within fp32 rounding of an integer, where the
  bilinear derivative is discontinuous (the two implementations pick different
  cells); every coarse-scale pixel aggregating one of them inherits the jump.  There
  the bar is on the relative L2 with the largest 0.1 % of the per-pixel differences
  left out (`trimmed_rel_l2`), per case and scale (FULL_T1 / FULL_T2), together with
  >= 98.5 % .. 99.9 % of pixels within 1e-4 max|ref| + 1e-3 |ref|;
* pose gradients (dL/daxisangle, dL/dtranslation, which sum over every pixel
  including the flipped ones): tier 2 <= 1e-4 small, 5e-3 full.
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


def trimmed_rel_l2(g, r, frac=1e-3):
    """relative L2 with the ceil(frac * n) largest absolute differences left out"""
    g = np.asarray(g, np.float64).ravel()
    r = np.asarray(r, np.float64).ravel()
    d = np.abs(g - r)
    n = int(np.ceil(frac * d.size))
    keep = np.ones(d.size, bool)
    if n:
        keep[np.argpartition(d, -n)[-n:]] = False
    return rel_l2(g[keep], r[keep])


def in_tol(g, r):
    return float((np.abs(g - r) <= 1e-4 * np.abs(r).max() + 1e-3 * np.abs(r)).mean())


SMALL_BAR = 1e-4          # tier 1 and tier 2 relative L2, small cases
# argmin differences vs the reference's (any candidate, not only identity vs
# reprojection): measured at most 1.3e-4 of the pixels per scale (1024x320, stereo)
FLIP_FRAC = 4e-4
# the one cell-flip pixel of stereo_b2_64x128 lands in the 8x16 scale 3 (measured 9.6e-4)
SMALL_T2_OVERRIDE = {("stereo_b2_64x128", 3): 3e-3}
# posecnn couples every pixel of a scale through T: the translation is scaled by the mean
# inverse depth of the scale (trainer.py:366-375), so dL/ddisp carries a uniform term
# proportional to dL/dT, a sum over the whole scale.  The reference's own fp32 run is
# 1.43e-3 from its fp64 run at the 8x16 scale 3 of posecnn_b2_64x128 and 3.1e-3 / 3.6e-3
# on the pose gradients (argmin pinned to the reference's; computed in the build
# container): bars 3 sqrt(2) x that floor there
_POSECNN_SMALL_FLOOR = {"posecnn_b2_64x128": {"disp": (2.02e-5, 2.11e-5, 1.63e-5, 1.43e-3),
                                              "axis": 3.07e-3, "trans": 3.55e-3}}


def small_bar(name, s, override=None):
    fl = _POSECNN_SMALL_FLOOR.get(name)
    bar = max(SMALL_BAR, _ceil2(3 * 2 ** 0.5 * fl["disp"][s])) if fl else SMALL_BAR
    return max(bar, (override or {}).get((name, s), 0.0))


def small_pose_bar(name, key, default):
    fl = _POSECNN_SMALL_FLOOR.get(name)
    return max(default, _ceil2(3 * 2 ** 0.5 * fl[key])) if fl else default
# per-scale bars on trimmed_rel_l2 for tier 1 (vs goldens outside the flip footprint;
# C2: vs the oracle, its golden holds checksums) and tier 2 (pinned oracle).  Round 4:
# anchored on the fp32 floor of the REFERENCE formulation, not on this implementation:
# F = the CPU-fp32 oracle's trimmed distance to the fp64 anchor (argmin pinned to the
# reference's; profiles/r04/parity_floor.json "cpu32_f64_trim", tests/
# test_parity_floor_gpu.py), bar = 3 * sqrt(2) * F rounded up — tiers 1/2 compare two
# fp32 implementations, each at most at the floor from the exact result, whose
# distance is then ~sqrt(2) F for independent rounding; k = 3 on that.
_FLOOR_TRIM = {"full_mono_b2_192x640": (5.78e-5, 7.36e-5, 9.50e-5, 9.12e-4),
               "full_mono_b2_320x1024": (1.10e-4, 2.01e-4, 1.48e-3, 4.41e-3),
               "full_stereo_b2_192x640": (6.25e-5, 7.07e-5, 8.56e-5, 9.48e-4),
               "c2_mono_b12_192x640": (6.57e-5, 9.32e-5, 6.81e-4, 2.54e-3),
               # round 5 (stereo-only S=1, posecnn per-scale T): the CPU-fp32 oracle's
               # trimmed distance to the fp64 anchor, computed in the build container
               "full_stereo_only_b2_192x640": (3.3e-5, 4.7e-5, 6.14e-4, 4.16e-3),
               "full_posecnn_b2_192x640": (5.32e-5, 1.36e-4, 9.07e-5, 3.03e-3)}
# posecnn at full size: the per-scale dL/dT (one scale's pixels, not the sum over scales)
# of the reference's own fp32 run is up to 8.7e-3 from the fp64 anchor (argmin pinned;
# computed in the build container), [scale][frame -1, 1]; bar 3 sqrt(2) x that floor
_POSECNN_T_FLOOR = {"full_posecnn_b2_192x640": ((2.93e-4, 8.29e-4), (8.31e-3, 1.33e-3), (8.50e-4, 2.36e-3),
                                                (3.12e-3, 8.74e-3))}
# tier 1 of the per-scale dL/dT (each implementation on its own argmin, against the
# golden): the larger of the reference formulation's distances on the host CPU and with
# ATen on the GPU, per (scale, temporal frame) — profiles/r06/parity_floor.json
# "grad_T_tier1" (tools/parity_floor.py; HIP measured 0.45-1.4x of it)
_POSECNN_T1_FLOOR = {"full_posecnn_b2_192x640": ((4.53e-3, 3.56e-3), (9.19e-3, 3.26e-3), (4.03e-3, 1.17e-2),
                                                 (3.10e-3, 1.16e-2))}
# the round-3 per-case bars (3x what HIP measured then): ADVICE r04 — the floor-anchored
# bar must not loosen a case below what the implementation was already held to, so each
# bar is the smaller of the two
_MEASURED_T1 = {"full_mono_b2_192x640": (2e-4, 2.5e-4, 3e-4, 1.6e-3),
                "full_mono_b2_320x1024": (2.5e-4, 3e-4, 2e-3, 7e-3),
                "full_stereo_b2_192x640": (2e-4, 2e-4, 4.5e-4, 4.5e-3),
                "c2_mono_b12_192x640": (2.5e-4, 1e-3, 6e-3, 1.2e-2)}
_MEASURED_T2 = {"full_mono_b2_192x640": (2e-4, 2.5e-4, 3e-4, 2e-3),
                "full_mono_b2_320x1024": (3e-4, 3.5e-4, 3.2e-3, 9.5e-3),
                "full_stereo_b2_192x640": (2e-4, 2.5e-4, 3e-4, 6e-3),
                "c2_mono_b12_192x640": (2.5e-4, 3.2e-4, 1.5e-3, 6.5e-3)}


def _ceil2(x):
    """x rounded UP to two significant digits"""
    e = 10.0 ** (np.floor(np.log10(x)) - 1)
    return float(np.ceil(x / e - 1e-9) * e)


_FLOOR_BAR = {n: tuple(_ceil2(3 * 2 ** 0.5 * f) for f in v) for n, v in _FLOOR_TRIM.items()}
FULL_T1 = {n: tuple(min(a, b) for a, b in zip(v, _MEASURED_T1.get(n, v))) for n, v in _FLOOR_BAR.items()}
FULL_T2 = {n: tuple(min(a, b) for a, b in zip(v, _MEASURED_T2.get(n, v))) for n, v in _FLOOR_BAR.items()}
# fraction of pixels within 1e-4 max|ref| + 1e-3 |ref| (measured >= 0.9857 at 1024x320 s3)
# (bar = 1 - 3x the measured out-of-tolerance fraction)
FULL_IN_TOL = (0.9998, 0.996, 0.987, 0.955)
# C2 gradient checksums vs the reference's, relative (3x measured): sum |g|, sum g^2,
# and sum |g| per image
CHECKSUM_BAR = {"abs": (1e-4, 1e-4, 4e-4, 7e-4), "sq": (2e-4, 1e-4, 4.5e-4, 1.2e-3)}
CHECKSUM_IMG_BAR = (6e-4, 1.1e-3, 2.2e-3, 4e-3)


def golden_flips(case, out, s):
    """HIP argmin != the reference's recorded argmin (None when the golden has none)"""
    if f"argmin_{s}" not in case.z.files:
        return None
    return out["select"][s] != case.expected(f"argmin_{s}")


def footprint_scale(case, s):
    return 0 if "v1_multiscale" in case.flags else s


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
    if case.checksums_only:
        # configs[1]'s shape (B=12, 640x192): the golden holds gradient checksums, the
        # per-pixel comparison is against the oracle on the regenerated inputs
        for s in range(4):
            g = out["grad_disp"][s].astype(np.float64)
            for key, v in (("abs", np.abs(g).sum()), ("sq", np.square(g).sum())):
                want = float(case.expected(f"grad_disp_{key}_{s}"))
                assert abs(v - want) <= CHECKSUM_BAR[key][s] * abs(want), (s, key, v, want)
            img = np.abs(g).sum((1, 2, 3))
            want = case.expected(f"grad_disp_abs_img_{s}")
            assert np.all(np.abs(img - want) <= CHECKSUM_IMG_BAR[s] * want), (s, img, want)
        cpu = run_oracle(case)
        for s in range(4):
            flips = golden_flips(case, out, s)
            assert flips.sum() <= max(3, FLIP_FRAC * flips.size), (s, int(flips.sum()))
            keep = ~flip_footprint(flips, s)
            e = trimmed_rel_l2(out["grad_disp"][s][keep], cpu["grad_disp"][s][keep])
            assert e <= FULL_T1[name][s], (s, e)
        return
    for s in range(4):
        want = case.expected(f"grad_disp_{s}")
        flips = golden_flips(case, out, s)
        keep = np.ones(want.shape, bool)
        if flips is not None:
            assert flips.sum() <= max(3, FLIP_FRAC * flips.size), (s, int(flips.sum()))
            keep = ~flip_footprint(flips, footprint_scale(case, s))
        if case.full:
            e = rel_l2(out["grad_disp"][s][keep], want[keep])
            assert e <= small_bar(name, s), (s, e)
        else:
            e = trimmed_rel_l2(out["grad_disp"][s][keep], want[keep])
            assert e <= FULL_T1[name][s], (s, e)
    # pose gradients sum over every pixel, flipped ones included (measured: small cases
    # <= 1.6e-4, stereo / full size <= 1.7e-3)
    if not case.temporal:   # stereo-only: T = stereo_T, no pose parameters
        return
    pose_bar = 5e-3 if (not case.full or name.startswith("stereo")) else 5e-4
    assert rel_l2(out["grad_axis"], case.expected("grad_axisangle")) <= small_pose_bar(name, "axis", pose_bar)
    assert rel_l2(out["grad_trans"], case.expected("grad_translation")) <= small_pose_bar(name, "trans", pose_bar)
    for i, f in enumerate(case.temporal):
        fi = case.frame_ids[1:].index(f)
        if case.posecnn:   # the per-scale T of trainer.py:374-375 and dL/dT at each scale
            for s in range(4):
                e = rel_l2(out["grad_T"][s][fi], case.expected(f"grad_T_{f}_{s}"))
                # unpinned: an argmin flip anywhere in the scale moves that scale's dL/dT,
                # so the bar is 3x the reference formulation's own unpinned distance to the
                # golden on the two fp32 platforms (_POSECNN_T1_FLOOR); the argmin-pinned
                # comparison (tier 2) holds it to 3 sqrt(2) x the pinned fp32 floor
                t1 = _POSECNN_T1_FLOOR.get(name)
                bar = _ceil2(3 * t1[s][i]) if t1 else small_pose_bar(name, "trans", pose_bar)
                assert e <= bar, (f, s, e, bar)
        else:
            assert rel_l2(out["grad_T"][fi], case.expected(f"grad_T_{f}")) <= pose_bar
    for s, g in out.get("grad_mask", {}).items():
        assert rel_l2(g, case.expected(f"grad_mask_{s}")) <= SMALL_BAR, (s, rel_l2(g, case.expected(f"grad_mask_{s}")))


@pytest.mark.parametrize("name", case_names())
def test_hip_gradients_match_oracle_pinned_selection(name):
    case = Case(name)
    cfg, out = run_hip(case)
    sel = None if cfg.disable_automasking and cfg.avg_reprojection else out["select"]
    ref = run_oracle(case, selection=sel)
    for s in range(5):
        assert abs(out["loss"][s] - ref["loss"][s]) <= 2e-6, (s, out["loss"][s], ref["loss"][s])
    small = name not in FULL_T2
    for s in range(4):
        g, r = out["grad_disp"][s], ref["grad_disp"][s]
        if small:
            e = rel_l2(g, r)
            assert e <= small_bar(name, s, SMALL_T2_OVERRIDE), (s, e)
        else:
            e = trimmed_rel_l2(g, r)
            assert e <= FULL_T2[name][s], (s, e)
            assert in_tol(g, r) >= FULL_IN_TOL[s], (s, in_tol(g, r))
    pose_bar = (6e-4 if name.startswith("stereo") else SMALL_BAR) if small else 5e-3
    if case.temporal:
        assert rel_l2(out["grad_axis"], ref["grad_axis"]) <= small_pose_bar(name, "axis", pose_bar)
        assert rel_l2(out["grad_trans"], ref["grad_trans"]) <= small_pose_bar(name, "trans", pose_bar)
    if case.posecnn and "T" in ref:   # the per-scale dL/dT, both sides on the HIP argmin
        for s in range(4):
            for i, f in enumerate(case.temporal):
                fi = case.frame_ids[1:].index(f)
                e = rel_l2(out["grad_T"][s][fi], ref["T"][s * len(case.temporal) + i])
                fl = _POSECNN_T_FLOOR.get(name)
                bar = max(pose_bar, _ceil2(3 * 2 ** 0.5 * fl[s][i])) if fl else small_pose_bar(name, "trans", pose_bar)
                assert e <= bar, (f, s, e, bar)
    for s, g in out.get("grad_mask", {}).items():
        assert rel_l2(g, ref["grad_mask"][s]) <= SMALL_BAR, s


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
        e = rel_l2(g, r)
        assert e <= SMALL_T2_OVERRIDE.get((name, s), SMALL_BAR), (s, e)
    pose_bar = 6e-4 if name.startswith("stereo") else SMALL_BAR
    assert rel_l2(out["grad_axis"], ref["grad_axis"]) <= pose_bar
    assert rel_l2(out["grad_trans"], ref["grad_trans"]) <= pose_bar
    # the warped colours the 8-bit gathers produce (generate_images reads fp32) agree
    # through the loss: an unpinned run selects the same candidates up to near-ties
    ref_free = run_oracle(case)
    C = cfg.num_src
    for s in range(4):
        flips = int(((out["select"][s] > C - 1)
                     != (ref_free["outputs"][f"identity_selection/{s}"].cpu().numpy() > 0.5)).sum())
        assert flips <= max(2, 1e-4 * out["select"][s].size), (s, flips)


@pytest.mark.parametrize("name", ["mono_b2_64x128", "stereo_b2_64x128"])
def test_caller_src8_matches_in_kernel_pack(name):
    """md2_tensors.src8: the sources' 8-bit RGBx copies handed in by the caller
    (data.pack_rgbx / md2_aug_run2) instead of packed by the forward — the same
    dwords, so the losses, the selection and every gradient are bitwise those of the
    in-kernel pack."""
    from monodepth2_amd.hotpath import photometric_loss
    from monodepth2_amd.data import pack_rgbx
    from hotpath_case import case_config, case_operands
    from monodepth2_amd.layers import transformation_from_parameters
    case = Case(name)
    for k, v in list(case.inputs.items()):
        if isinstance(k, tuple) and k[0] in ("color", "color_aug"):
            case.inputs[k] = torch.round(v * 255.0) / 255.0
    cfg = case_config(case)
    colors, K, inv_K, noise = case_operands(case, "cuda")
    Ts, ti = [], 0
    for f in case.frame_ids[1:]:
        if f == "s":
            Ts.append(case.inputs["stereo_T"].cuda())
        else:
            Ts.append(transformation_from_parameters(case.axisangle[ti].cuda(), case.translation[ti].cuda(),
                                                     invert=(f < 0)))
            ti += 1
    src8 = pack_rgbx([colors[0][fi] for fi in range(1, cfg.num_src + 1)])
    res = []
    for s8 in (None, src8):
        T = torch.stack(Ts).detach().requires_grad_(True)
        disps = [case.disps[s].cuda().requires_grad_(True) for s in range(4)]
        loss, sel = photometric_loss(cfg, disps, colors, K, inv_K, T, noise=noise, src8=s8)
        loss[cfg.num_scales].backward()
        torch.cuda.synchronize()
        res.append((loss.clone(), sel.clone(), [d.grad.clone() for d in disps], T.grad.clone()))
    (l0, s0, g0, t0), (l1, s1, g1, t1) = res
    assert torch.equal(l0, l1) and torch.equal(s0, s1) and torch.equal(t0, t1)
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))
    with pytest.raises(ValueError, match="src8"):
        photometric_loss(cfg, [case.disps[s].cuda() for s in range(4)], colors, K, inv_K,
                         torch.stack(Ts).detach(), noise=noise, src8=src8[:, :1].contiguous())


@pytest.mark.parametrize("name", ["mono_b2_64x128", "stereo_b2_64x128"])
def test_bf16_disparities_read_directly(name):
    """md2_desc.disp_dtype = bf16 (the depth decoder's output under bf16 autocast, C5):
    the kernels read the bf16 disparities as is.  bf16 -> fp32 is exact, so the losses
    and the selection equal those of the same values cast up to fp32, bit for bit, and
    the gradients the kernel writes in bf16 are the fp32 path's rounded to nearest even
    (what the cast-up's autograd backward returns)."""
    from monodepth2_amd.hotpath import photometric_loss
    from hotpath_case import case_config, case_operands
    from monodepth2_amd.layers import transformation_from_parameters
    case = Case(name)
    cfg = case_config(case)
    colors, K, inv_K, noise = case_operands(case, "cuda")
    base = [case.disps[s].cuda().to(torch.bfloat16) for s in range(4)]
    Ts = []
    ti = 0
    for f in case.frame_ids[1:]:
        if f == "s":
            Ts.append(case.inputs["stereo_T"].cuda())
        else:
            Ts.append(transformation_from_parameters(case.axisangle[ti].cuda(), case.translation[ti].cuda(),
                                                     invert=(f < 0)))
            ti += 1
    T = torch.stack(Ts).detach()
    out = {}
    for dt in (torch.bfloat16, torch.float32):
        d = [b.detach().to(dt).clone().requires_grad_(True) for b in base]
        Tg = T.clone().requires_grad_(True)
        loss, sel = photometric_loss(cfg, d, colors, K, inv_K, Tg, noise=noise)
        loss[4].backward()
        out[dt] = (loss.detach().cpu(), sel.cpu(), [x.grad for x in d], Tg.grad.cpu())
    lb, sb, gb, tb = out[torch.bfloat16]
    lf, sf, gf, tf = out[torch.float32]
    assert torch.equal(lb, lf) and torch.equal(sb, sf)
    for s in range(4):
        assert gb[s].dtype == torch.bfloat16
        assert torch.equal(gb[s], gf[s].to(torch.bfloat16)), s
    assert torch.equal(tb, tf)
