#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for c in 0 6 12 24; do
    MD2_X6_SPLIT_COST=$c timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity > gpurun_out/abs.log 2>&1 || exit 1
    echo "cost $c: $(grep -o 'timed: [0-9.]* ms/step' gpurun_out/abs.log) $(grep -o 'host enqueue time: [0-9.]* ms/step' gpurun_out/abs.log)"
  done
done
