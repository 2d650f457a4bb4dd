#!/bin/bash
# Session-3 GPU call: -m gpu tests, default bench, same-box step A/B against the
# session-start tree (variants/h0, a built worktree), x6 conv micro A/B, per-step trace.
set -o pipefail
mkdir -p gpurun_out/s3 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/tests.log 2>&1 || exit 1
echo tests ok
timeout -k 10 300 python bench.py > gpurun_out/s3/bench_default.log 2>&1 || exit 1
echo bench ok
for i in 1 2; do
  for t in variants/h0 .; do
    (cd $t && timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity --pmc 0 --no-conv-roofline) \
        > gpurun_out/s3/abt_${i}_$(basename $t).log 2>&1 || exit 1
    echo "$t: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s3/abt_${i}_$(basename $t).log)" >> gpurun_out/s3/ab_tree.txt
  done
done
echo abtree ok
for v in wbase2 wnew2; do
  echo "== $v" >> gpurun_out/s3/ab_conv.log
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 5 200 python tools/conv_x6_bench.py s3 >> gpurun_out/s3/ab_conv.log 2>&1 || exit 1
done
echo abconv ok
bash tools/step_trace.sh s3trace > /dev/null 2>&1 || exit 1
echo trace ok
