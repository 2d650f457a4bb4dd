"""The fp32 parity floor at full size (tests/test_parity_floor_gpu.py's numbers, plus
ATen-on-GPU): per case and scale, relative L2 (untrimmed and with the largest 0.1 %
of differences left out) of dL/ddisp_s against the fp64 anchor for
  hip    the HIP path (its own argmin; flips vs the reference excluded with footprint)
  cpu32  the reference formulation in fp32 on the host CPU (oracle, argmin pinned)
  aten   the same ATen formulation in fp32 on PyTorch-ROCm (argmin pinned)
Run on the GPU box:  python tools/parity_floor.py profiles/r06/parity_floor.json
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

from golden_io import Case  # noqa: E402
from hotpath_case import run_hip, run_oracle  # noqa: E402
from test_hotpath_gpu import rel_l2  # noqa: E402
from test_parity_floor_gpu import K_FLOOR, floor_metrics, floor_runs, fp64_cases  # noqa: E402


def main():
    torch.set_num_threads(16)
    res = {"k_floor": K_FLOOR, "floor": "max over the reference formulation's fp32 runs (host CPU, ATen on the GPU) "
                                        "of the distance to the fp64 anchor; argmin pinned to the reference's",
           "cases": {}}
    for name in fp64_cases():
        case = Case(name)
        _, out = run_hip(case)
        r64, runs = floor_runs(case, out["select"] if case.posecnn else None)
        rows = floor_metrics(case, out, runs, r64)
        for row in rows:
            row["hip_over_floor"] = row["hip_f64"] / row["floor"]
            row["hip_over_floor_trim"] = row["hip_f64_trim"] / row["floor_trim"]
            print(name, {k: (round(v, 7) if isinstance(v, float) else v) for k, v in row.items()}, flush=True)
        pose = {k: {"hip_f64": rel_l2(out[k], r64[k]), **{f"{n}_f64": rel_l2(v[k], r64[k]) for n, v in runs.items()}}
                for k in ("grad_axis", "grad_trans")}
        loss = {"hip_minus_f64": [float(out["loss"][s] - r64["loss"][s]) for s in range(5)],
                **{f"{n}_minus_f64": [v["loss"][s] - r64["loss"][s] for s in range(5)] for n, v in runs.items()}}
        res["cases"][name] = {"scales": rows, "pose": pose, "loss": loss}
        if case.posecnn:
            # tier 1 of tests/test_hotpath_gpu.py: the per-scale dL/dT against the golden
            # (the reference's own fp32 run), each implementation on its OWN argmin — the
            # HIP path and the reference formulation on the two fp32 platforms
            own = {"cpu32": run_oracle(case), "aten": run_oracle(case, device="cuda")}
            t1 = []
            for s in range(4):
                for i, f in enumerate(case.temporal):
                    fi = case.frame_ids[1:].index(f)
                    want = case.expected(f"grad_T_{f}_{s}")
                    row = {"scale": s, "frame": f, "hip": rel_l2(out["grad_T"][s][fi], want)}
                    for n, v in own.items():
                        row[n] = rel_l2(v["T"][s * len(case.temporal) + i], want)
                    t1.append(row)
                    print(name, "dL/dT tier 1", row, flush=True)
            res["cases"][name]["grad_T_tier1"] = t1
    if len(sys.argv) > 1:
        os.makedirs(os.path.dirname(sys.argv[1]), exist_ok=True)
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
