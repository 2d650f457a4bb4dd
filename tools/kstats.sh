#!/bin/bash
# Per-kernel average GPU time of any command: bash tools/kstats.sh <tag> <command...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
mkdir -p $R/gpurun_out/$tag && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$tag/prof -o k --output-format csv -- "$@" \
  > $R/gpurun_out/$tag/run.log 2>&1 || { tail -5 $R/gpurun_out/$tag/run.log; exit 1; }
grep -v "^\[" $R/gpurun_out/$tag/run.log | tail -4
f=$(find $R/gpurun_out/$tag/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    n = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Name"]).split("(")[0]
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>4}  {n[:90]}")
PY
rm -f $(find $R/gpurun_out/$tag/prof -name "*kernel_trace.csv")
