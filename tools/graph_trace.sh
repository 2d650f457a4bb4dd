#!/bin/bash
# Kernel traces of the eager and the hipGraph-replayed bf16 B=32 step (C5), for
# tools/trace_timeline.py.
set -o pipefail
mkdir -p gpurun_out/gtrace && export TMPDIR=/tmp
for g in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gtrace/g$g -o run -- \
     python bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-parity --amp bf16 --batch 32 --graph $g \
     > gpurun_out/gtrace/g$g.log 2>&1 || exit 1
done
