"""Summarise rocprofv3 counter_collection CSVs: per kernel, average counter value per
dispatch.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KB;
on gfx950 FETCH_SIZE under-reports wide streaming reads by 2x (reported as
`fetch_bytes_x2`, an upper estimate for our 4-B-per-lane reads).

    python tools/pmc_summary.py out.json file1.csv [file2.csv ...]
"""
import collections
import csv
import json
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0]


def main():
    out_path, files = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in agg.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d:
            d["fetch_bytes"] = d["FETCH_SIZE"] * 1024
            d["fetch_bytes_x2"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024
        res[k] = d
    json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)
    for k, d in sorted(res.items()):
        print(k, {c: (round(v, 1) if isinstance(v, float) else v) for c, v in d.items()})


if __name__ == "__main__":
    main()
