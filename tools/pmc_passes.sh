#!/bin/bash
# Two counter passes (issue/occupancy, memory units) over any command, summarised per
# kernel:  bash tools/pmc_passes.sh <tag> <kernel-regex> <command...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; rx=$2; shift 2
out=$R/gpurun_out/$tag
mkdir -p $out && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
i=1
for C in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$rx" -d $out/p$i -o pmc --output-format csv -- "$@" \
    > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
  i=$((i+1))
done
python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    g = m.get("GRBM_GUI_ACTIVE", 1)
    print(k[:60], {c: round(v) for c, v in m.items()})
    cyc = g / 8.0   # kernel cycles (GRBM_GUI_ACTIVE summed over the 8 XCDs)
    print("   per-CU-unit busy: td", round(m.get("TD_TD_BUSY_sum", 0) / 256 / cyc, 3), "ta",
          round(m.get("TA_TA_BUSY_sum", 0) / 256 / cyc, 3), "| valu insts per SIMD-cycle",
          round(m.get("SQ_INSTS_VALU", 0) / 1024 / cyc, 3), "| wait/wave-cycles",
          round(m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1)), 3))
PY
