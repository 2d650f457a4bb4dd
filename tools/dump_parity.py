"""Dump HIP and oracle (HIP-pinned selection) gradients of one golden case to
gpurun_out/dump_<case>.npz for offline analysis.

    python tools/dump_parity.py <case>
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

from golden_io import Case  # noqa: E402
from hotpath_case import run_hip, run_oracle  # noqa: E402


def main():
    name = sys.argv[1]
    case = Case(name)
    cfg, out = run_hip(case)
    ref = run_oracle(case, selection=out["select"])
    rec = {}
    for s in range(4):
        rec[f"hip_{s}"] = out["grad_disp"][s]
        rec[f"ora_{s}"] = ref["grad_disp"][s]
        rec[f"sel_{s}"] = np.asarray(out["select"][s])
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, "gpurun_out", f"dump_{name}.npz"), **rec)
    print("ok")


if __name__ == "__main__":
    main()
