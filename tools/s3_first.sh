#!/bin/bash
# Session-3 first GPU call: -m gpu tests, default bench, x6 wgrad layout A/B, per-step trace.
set -o pipefail
mkdir -p gpurun_out/s3 && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/tests.log 2>&1 || exit 1
echo tests ok
timeout -k 10 300 python bench.py > gpurun_out/s3/bench_default.log 2>&1 || exit 1
echo bench ok
for v in wbase2 wnew2 wbase2 wnew2; do
  echo "== $v" >> gpurun_out/s3/ab_wgrad.log
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 5 200 python tools/conv_x6_bench.py quickw >> gpurun_out/s3/ab_wgrad.log 2>&1 || exit 1
  echo "== $v" >> gpurun_out/s3/ab_fwd.log
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 5 200 python tools/conv_x6_bench.py quick >> gpurun_out/s3/ab_fwd.log 2>&1 || exit 1
done
echo ab ok
bash tools/step_trace.sh s3trace > /dev/null 2>&1 || exit 1
echo trace ok
