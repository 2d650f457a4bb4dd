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
"""
import numpy as np
import pytest
import torch

from golden_io import Case, case_names
from hotpath_case import run_hip, run_oracle

pytestmark = pytest.mark.gpu


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
    ref = run_oracle(case, selection=None if cfg.disable_automasking and cfg.avg_reprojection else out["select"])
    for s in range(5):
        assert abs(out["loss"][s] - ref["loss"][s]) <= 2e-6, (s, out["loss"][s], ref["loss"][s])
    for s in range(4):
        g, r = out["grad_disp"][s], ref["grad_disp"][s]
        ok = np.abs(g - r) <= 1e-4 * np.abs(r).max() + 1e-3 * np.abs(r)
        assert ok.mean() >= 0.99, (s, ok.mean())
        assert rel_l2(g, r) <= 1e-2, (s, rel_l2(g, r))
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
