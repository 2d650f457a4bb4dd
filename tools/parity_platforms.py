"""How far the HIP path and the reference's own ATen formulation on PyTorch-ROCm
each drift from the CPU oracle, argmin pinned to the HIP selection (no asserts).

    python tools/parity_platforms.py [case ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

from golden_io import Case, case_names  # noqa: E402
from hotpath_case import run_hip, run_oracle  # noqa: E402


def metrics(g, r):
    ok = np.abs(g - r) <= 1e-4 * np.abs(r).max() + 1e-3 * np.abs(r)
    rel = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30))
    return float(ok.mean()), rel


def main():
    for name in sys.argv[1:] or case_names():
        case = Case(name)
        cfg, out = run_hip(case)
        sel = None if cfg.disable_automasking and cfg.avg_reprojection else out["select"]
        cpu = run_oracle(case, selection=sel)
        gpu = run_oracle(case, selection=sel, device="cuda")
        line = [f"{name:28s}"]
        for s in range(4):
            h = metrics(out["grad_disp"][s], cpu["grad_disp"][s])
            a = metrics(gpu["grad_disp"][s], cpu["grad_disp"][s])
            line.append(f"s{s} hip {h[0]:.4f}/{h[1]:.1e} aten-gpu {a[0]:.4f}/{a[1]:.1e}")
        print(" | ".join(line), flush=True)
        cpu_u = run_oracle(case)
        gpu_u = run_oracle(case, device="cuda")
        line = [f"{'  unpinned vs golden':28s}"]
        for s in range(4):
            want = case.expected(f"grad_disp_{s}")
            h = metrics(out["grad_disp"][s], want)
            a = metrics(gpu_u["grad_disp"][s], want)
            fl_h = fl_a = -1
            if not cfg.disable_automasking:
                C = 1 if cfg.avg_reprojection else cfg.num_src
                ref_sel = cpu_u["outputs"][f"identity_selection/{s}"].cpu().numpy() > 0.5
                fl_h = int(((out["select"][s] > C - 1) != ref_sel).sum())
                fl_a = int(((gpu_u["outputs"][f"identity_selection/{s}"].cpu().numpy() > 0.5) != ref_sel).sum())
            c = metrics(cpu_u["grad_disp"][s], want)
            line.append(f"s{s} hip {h[1]:.1e} flips {fl_h} aten-gpu {a[1]:.1e} flips {fl_a} host-cpu {c[1]:.1e}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
