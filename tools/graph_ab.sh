#!/bin/bash
# eager vs hipGraph step, pose network on its own stream or not (bf16 B=32, C5's per-GPU shape)
set -o pipefail
mkdir -p gpurun_out/gab && export TMPDIR=/tmp
run() { tag=$1; shift
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity "$@" > gpurun_out/gab/$tag.log 2>&1 || exit 1
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gab/$tag.log) $(grep -o 'host enqueue time: [0-9.]*' gpurun_out/gab/$tag.log)"
}
run e1 --amp bf16 --batch 32 --graph 0 --pose-stream 1
run g1 --amp bf16 --batch 32 --graph 1 --pose-stream 1
run e0 --amp bf16 --batch 32 --graph 0 --pose-stream 0
run g0 --amp bf16 --batch 32 --graph 1 --pose-stream 0
MD2_GRAPH_DOT=gpurun_out/gab/g1.dot run g1dot --amp bf16 --batch 32 --graph 1 --pose-stream 1 --steps 2
run f_e1 --graph 0
run f_g1 --graph 1
