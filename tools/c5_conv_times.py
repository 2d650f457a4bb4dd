"""Config C5's convolutions (bf16 autocast, B=32 640x192): the per-shape autotune times
of the bf16 GEMMs and MIOpen (conv_ops._times after two eager steps), sorted by the kept
candidate's time, and their sum per op — where the bf16 step's convolution time goes.

    python tools/c5_conv_times.py [--batch 32] [--amp bf16|none] [--out path.json]

With --amp none: the fp32 step's x6 / f32 / direct candidates instead (configs[1]: --batch 12).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from monodepth2_amd import conv_ops  # noqa: E402
from monodepth2_amd.data import synthetic_batch  # noqa: E402
from monodepth2_amd.options import default_options  # noqa: E402
from monodepth2_amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--amp", default="bf16", choices=["bf16", "none"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.manual_seed(0)
    tr = Trainer(default_options(batch_size=a.batch, height=192, width=640, weights_init="scratch",
                                 log_dir="/tmp/md2_c5t", frame_ids=[0, -1, 1], amp=a.amp), device=torch.device("cuda", 0))
    batch = synthetic_batch(a.batch, 192, 640, tr.opt.frame_ids, 4, seed=3, device="cuda", eight_bit=True)
    for _ in range(2):
        tr.train_step(batch)
    torch.cuda.synchronize()
    rows, tot = [], {}
    for k, i in conv_ops._choice.items():
        names = conv_ops._names.get(k)
        t = conv_ops._times.get(k, {})
        if names is None or k[0].endswith("bf16") != (a.amp == "bf16"):
            continue
        kept = names[i]
        rows.append({"op": k[0], "x": list(k[1]), "w": list(k[2]), "stride": k[3], "pad": k[4], "kept": kept,
                     "ms": {n: round(v, 4) for n, v in t.items()}})
        tot.setdefault(k[0], [0.0, 0.0])
        tot[k[0]][0] += t.get(kept, 0.0)
        tot[k[0]][1] += t.get("miopen", float("nan"))
    rows.sort(key=lambda r: -r["ms"].get(r["kept"], 0.0))
    for r in rows:
        print(r["op"], r["x"], r["w"], r["stride"], "kept", r["kept"], r["ms"])
    print("sum of kept / miopen ms per op (one call per shape):", {k: [round(v[0], 3), round(v[1], 3)] for k, v in tot.items()})
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"rows": rows, "sum_kept_vs_miopen_ms": tot}, f, indent=1)


if __name__ == "__main__":
    main()
