#!/bin/bash
# tests (given files) + eager/graph bench lines; usage: tools/gpu_step.sh <tag> [test files]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$tag/tests.log 2>&1 || { tail -30 gpurun_out/$tag/tests.log; exit 1; }
  tail -3 gpurun_out/$tag/tests.log
fi
run() { t=$1; shift
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity "$@" > gpurun_out/$tag/$t.log 2>&1 || exit 1
  echo "$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$tag/$t.log) $(grep -o 'host enqueue time: [0-9.]*' gpurun_out/$tag/$t.log)"
}
if [ -z "$NOBENCH" ]; then
run e32 --amp bf16 --batch 32 --graph 0
run g32 --amp bf16 --batch 32 --graph 1
run e12 --graph 0
run g12 --graph 1
fi
