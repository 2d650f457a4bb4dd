#!/bin/bash
# per-kernel times of the hot path alone (tools/hot_bench.py, configs[1] shape, 8-bit colours)
set -o pipefail
tag=${1:-hp}
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o hot --output-format csv -- python tools/hot_bench.py --eight-bit --iters 30 > gpurun_out/$tag/hot_bench.log 2>&1 || exit 1
tail -1 gpurun_out/$tag/hot_bench.log
f=$(find gpurun_out/$tag/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Name"]).split("(")[0]
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>4}  {n[:70]}")
PY
