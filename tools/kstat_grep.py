"""Calls / average duration of the kernels whose name contains a pattern, from rocprofv3
--stats kernel_stats.csv files.   python tools/kstat_grep.py PATTERN FILE..."""
import csv
import re
import sys

for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        if sys.argv[1] in r["Name"]:
            n = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Name"]).split("(")[0]
            print("%-60s %-45s calls %5s avg %8.1f us" % (path[-45:], n, r["Calls"], float(r["AverageNs"]) / 1000))
