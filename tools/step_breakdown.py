"""Per-step kernel time breakdown from a rocprofv3 kernel trace: steps are delimited by
the Adam kernel (one per training step); the last N steps are summed per kernel and
grouped (conv / bn / photometric / other).
    python tools/step_breakdown.py TRACE.csv [--last 20]"""
import argparse
import collections
import csv
import re


def group(name):
    n = name
    if "photo" in n or "md2hot" in n or "disp_grad_T" in n or "finalize" in n or "pack_src8" in n:
        return "photometric"
    if n.startswith("void (anonymous namespace)::bn_") or "(anonymous namespace)::bn_" in n:
        return "batchnorm"
    if "conv" in n or "stem" in n or "igemm" in n or "gemm" in n.lower() or "Cijk" in n or "naive" in n:
        return "conv"
    if "head_" in n:
        return "disp heads"
    if "pool" in n:
        return "maxpool"
    if "pad_" in n or "bias_act" in n or "upsample" in n:
        return "decoder glue"
    if "adam" in n:
        return "adam"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    steps = list(zip(adam[-a.last - 1:-1], adam[-a.last:]))
    per = collections.Counter()
    calls = collections.Counter()
    wall = 0.0
    for s, e in steps:
        wall += (int(rows[e]["End_Timestamp"]) - int(rows[s]["End_Timestamp"])) / 1e6
        for r in rows[s + 1:e + 1]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            per[r["Kernel_Name"]] += d
            calls[r["Kernel_Name"]] += 1
    n = len(steps)
    tot = sum(per.values()) / n
    print("steps %d: kernel time %.3f ms/step, adam-to-adam wall %.3f ms/step" % (n, tot, wall / n))
    g = collections.Counter()
    for k, v in per.items():
        g[group(k)] += v / n
    for k, v in g.most_common():
        print("  %-14s %7.3f ms" % (k, v))
    print()
    for k, v in per.most_common(30):
        print("%7.3f ms  %5.1f calls  %7.1f us avg  %s" % (v / n, calls[k] / n, v / calls[k] * 1e3, re.sub(r"\(anonymous namespace\)::", "", k)[:100]))


if __name__ == "__main__":
    main()
