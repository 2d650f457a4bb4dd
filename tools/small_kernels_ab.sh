#!/bin/bash
# The hot path's small kernels (smoothness forward, dL/d(disp) + dL/dT tail, finalize,
# pack) under two library builds on one box: per-kernel average times from a
# rocprofv3 kernel trace of tools/hot_bench.py, then one PMC pass each.
#   bash tools/small_kernels_ab.sh <tag> <variant> <variant> ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
for v in "$@"; do
  d=gpurun_out/$tag/$v$rep
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o k --output-format csv \
    -- python3 tools/hot_bench.py --eight-bit --iters 30 > $d.log 2>&1 || exit 1
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "== $v rep $rep: $(tail -1 $d.log)"
  python3 - "$f" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Name"]).split("(")[0]
    if re.search("photo_|smooth|disp_grad|grad_T|finalize|pack_src8", n):
        print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>4}  {n[:60]}")
PY
  rm -f $(find $d -name "*kernel_trace.csv")
done
done
