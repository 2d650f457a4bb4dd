#!/bin/bash
# Kernel trace of an eager bench run + per-step breakdown: bash tools/step_trace.sh <tag> [family ...]
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$tag && export TMPDIR=/tmp
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$tag/t -o s --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --graph ${GRAPH:-0} --no-conv-roofline \
  > gpurun_out/$tag/log 2>&1 || exit 1
python3 tools/trace_breakdown.py gpurun_out/$tag/t/s_kernel_trace.csv 20 "$@" > gpurun_out/$tag/breakdown.txt
rm -f gpurun_out/$tag/t/s_kernel_trace.csv
cat gpurun_out/$tag/breakdown.txt
