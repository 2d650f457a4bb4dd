"""Print HIP-vs-reference parity numbers for every golden case (no asserts).

    python tools/parity_report.py [case ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

from golden_io import Case, case_names  # noqa: E402
from hotpath_case import run_hip  # noqa: E402


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def main():
    names = sys.argv[1:] or case_names()
    for name in names:
        case = Case(name)
        cfg, out = run_hip(case)
        dl = max(abs(out["loss"][s] - float(case.expected(f"loss_{s}"))) for s in range(4))
        dl = max(dl, abs(out["loss"][4] - float(case.expected("loss"))))
        gd = [rel_l2(out["grad_disp"][s], case.expected(f"grad_disp_{s}")) for s in range(4)]
        ga = rel_l2(out["grad_axis"], case.expected("grad_axisangle"))
        gt = rel_l2(out["grad_trans"], case.expected("grad_translation"))
        line = f"{name:28s} loss|d|={dl:.1e} gdisp={' '.join(f'{e:.1e}' for e in gd)} gaxis={ga:.1e} gtrans={gt:.1e}"
        if case.full:
            wmax = 0.0
            for s in range(4):
                for fi, f in enumerate(case.frame_ids[1:]):
                    wmax = max(wmax, float(np.abs(out["gen"]["color"][(fi, s)].cpu().numpy()
                                                  - case.expected(f"warp_{f}_{s}")).max()))
            line += f" warp|d|max={wmax:.1e}"
            if "disable_automasking" not in case.flags:
                C = 1 if cfg.avg_reprojection else cfg.num_src
                flips = [int(((out["select"][s] > C - 1).astype(np.uint8)
                              != case.expected(f"identity_selection_{s}")).sum()) for s in range(4)]
                line += f" selflips={flips}"
        print(line, flush=True)
        if "--dump" in os.environ.get("MD2_PARITY", ""):
            np.savez(os.path.join(REPO, "gpurun_out", f"parity_{name}.npz"),
                     **{f"gd{s}": out["grad_disp"][s] for s in range(4)},
                     **{f"sel{s}": out["select"][s] for s in range(4)})


if __name__ == "__main__":
    main()
