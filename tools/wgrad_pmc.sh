#!/bin/bash
# Counter passes over one weight-gradient shape per variant (tools/wgrad_one.py):
#   bash tools/wgrad_pmc.sh <tag> "B Cin Cout pad H W" flags...
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
tag=$1; shape=$2; shift 2
out=$R/gpurun_out/$tag
mkdir -p $out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS TA_TA_BUSY_sum TD_TD_BUSY_sum"
for fl in "$@"; do
  for pi in 1 2; do
    if [ $pi = 1 ]; then C=$P1; else C=$P2; fi
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "conv_x6" -d $out/f${fl}_p$pi -o pmc --output-format csv -- \
      python3 $R/tools/wgrad_one.py $shape $fl 10 > $out/f${fl}_p$pi.log 2>&1
  done
done
python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(os.path.relpath(f, out).split("/")[0], k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
