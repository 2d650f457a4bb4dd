#!/bin/bash
# Session-3: BatchNorm ReLU-mask backward (ABI 15) — GPU tests, same-box step A/B vs the
# previous commit (variants/h1, a built worktree), default bench.
set -o pipefail
mkdir -p gpurun_out/s3 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/tests_bn.log 2>&1 || exit 1
echo tests ok
for i in 1 2; do
  for t in variants/h1 .; do
    (cd $t && timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity --pmc 0 --no-conv-roofline) \
        > gpurun_out/s3/abbn_${i}_$(basename $t).log 2>&1 || exit 1
    echo "$t: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s3/abbn_${i}_$(basename $t).log)" >> gpurun_out/s3/ab_bn.txt
  done
done
echo ab ok
timeout -k 10 300 python bench.py > gpurun_out/s3/bench_bn.log 2>&1 || exit 1
echo bench ok
