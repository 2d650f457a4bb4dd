#!/bin/bash
# One GPU round trip: selected -m gpu tests, a rocprofv3 kernel trace of the bench,
# and a plain bench line.  Usage: tools/gpu_check.sh <tag> [test files...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out && export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/${tag}_tests.log 2>&1 || exit 1
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run -- python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity > gpurun_out/prof_${tag}.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/bench_${tag}.log 2>&1
