"""Per-step GPU time by kernel (and by launch shape for chosen families) from a
rocprofv3 --kernel-trace csv of an eager bench run: the last `steps` steps, split at
the photometric forward's first kernel (photo_ident; pack_src8 before round 3).
    python tools/trace_breakdown.py <kernel_trace.csv> [steps] [family ...]"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    fams = sys.argv[3:]
    rows = list(csv.DictReader(open(path)))
    names = [r["Kernel_Name"] for r in rows]
    marks = [i for i, n in enumerate(names) if "photo_ident" in n] or \
        [i for i, n in enumerate(names) if "pack_src8" in n]
    sel = rows[marks[-steps]:]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    shp = collections.defaultdict(list)
    for r in sel:
        n = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Kernel_Name"]).split("(")[0]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[n][0] += 1
        agg[n][1] += d
        if any(f in n for f in fams):
            shp[(n[:60], r["Grid_Size_X"], r["Grid_Size_Y"])].append(d)
    tot = sum(v[1] for v in agg.values())
    print(f"span {(t1 - t0) / 1e6 / steps:.3f} ms/step, kernel sum {tot / 1e6 / steps:.3f} ms/step")
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{d / 1e6 / steps:7.3f} ms {c / steps:6.1f}/step  {n[:110]}")
    for k, v in sorted(shp.items(), key=lambda kv: -sum(kv[1]))[:40]:
        print(f"  {sum(v) / steps / 1e3:7.1f} us/step n={len(v) / steps:4.1f} avg {sum(v) / len(v) / 1e3:6.1f} us "
              f"grid {k[1]}x{k[2]}  {k[0]}")


if __name__ == "__main__":
    main()
