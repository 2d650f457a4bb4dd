"""Compare hot_bench.py --dump files: bitwise equality and the largest relative
difference per tensor (A/B of library builds run with MD2_LIB).

    python tools/cmp_dumps.py REF.pt OTHER.pt [OTHER2.pt ...]
"""
import sys

import torch


def flat(d):
    out = {"loss": d["loss"], "T": d["T"]}
    for s, g in enumerate(d["disps"]):
        out[f"disp{s}"] = g
    return out


def main():
    ref = flat(torch.load(sys.argv[1], weights_only=True))
    for p in sys.argv[2:]:
        o = flat(torch.load(p, weights_only=True))
        same = all(torch.equal(ref[k], o[k]) for k in ref)
        rel = {k: float((ref[k] - o[k]).norm() / ref[k].norm().clamp_min(1e-30)) for k in ref}
        print(p, "bitwise" if same else "DIFFERS", {k: f"{v:.2e}" for k, v in rel.items()})


if __name__ == "__main__":
    main()
