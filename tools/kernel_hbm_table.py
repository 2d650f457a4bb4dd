"""Per-kernel HBM roofline table of the hand-written kernels: average duration (the
round's --stats trace), HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes
(tools/hbm_table.sh; KB -> B, reads x2 per MI355X_MICROARCH.md's gfx950 FETCH_SIZE
correction: an upper estimate), achieved GB/s and the fraction of 8 TB/s.
    python tools/kernel_hbm_table.py r01   ->  profiles/r01/kernel_hbm.json + a markdown table"""
import collections
import csv
import glob
import json
import os
import re
import sys

PEAK = 8000.0   # GB/s


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"^void ", "", n).split("(")[0]


def main():
    rnd = sys.argv[1]
    src = os.path.join("gpurun_out", rnd)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))[0]
    dur = {}
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        dur.setdefault(k, [0.0, 0])
        dur[k][0] += float(r["TotalDurationNs"])
        dur[k][1] += int(r["Calls"])
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "hbm*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            cnt[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, cs in cnt.items():
        if k not in dur or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        avg_ns = dur[k][0] / dur[k][1]
        rd = 2 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
        wr = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        gbs = (rd + wr) / avg_ns
        rows.append({"kernel": k, "calls_in_trace": dur[k][1], "avg_us": round(avg_ns / 1e3, 2),
                     "us_per_step_share": round(dur[k][0] / 1e3, 1),
                     "hbm_read_mb": round(rd / 1e6, 2), "hbm_write_mb": round(wr / 1e6, 2),
                     "gbs": round(gbs, 1), "frac_of_8tbs": round(gbs / PEAK, 3)})
    rows.sort(key=lambda r: -r["us_per_step_share"])
    dst = os.path.join("profiles", rnd, "kernel_hbm.json")
    json.dump(rows, open(dst, "w"), indent=1)
    print("| kernel | avg µs | HBM MB/launch (r+w) | GB/s | of 8 TB/s |")
    print("|---|---|---|---|---|")
    for r in rows:
        print(f"| `{r['kernel']}` | {r['avg_us']} | {r['hbm_read_mb']}+{r['hbm_write_mb']} | {r['gbs']} | "
              f"{r['frac_of_8tbs']:.2f} |")


if __name__ == "__main__":
    main()
