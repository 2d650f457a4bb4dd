#!/bin/bash
# per-kernel times of the hot path for several variant builds (tools/build_variant.sh)
#   tools/ab_prof.sh tag name1 name2 ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
for v in "$@"; do
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/$v -o hot --output-format csv -- python tools/hot_bench.py --eight-bit --iters 30 > gpurun_out/$tag/$v.log 2>&1 || exit 1
  f=$(find gpurun_out/$tag/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v $(tail -1 gpurun_out/$tag/$v.log)"
  python - "$f" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(anonymous namespace\)::|^void ", "", r["Name"]).split("(")[0]
    if any(t in n for t in ("photo_", "disp_grad", "pack_src8", "smooth_fwd", "finalize", "grad_T")):
        print(f"{float(r['AverageNs'])/1e3:9.1f} us  {n[:60]}")
PY
done
