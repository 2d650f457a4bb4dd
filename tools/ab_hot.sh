#!/bin/bash
# A/B the photometric kernels of several variant builds (tools/build_variant.sh):
#   tools/ab_hot.sh name1 name2 ...   (run on the GPU box from the repo root)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  echo -n "$v: "
  MD2_LIB=variants/$v/libmd2hot.so timeout -k 5 120 python tools/hot_bench.py --iters 40 ${HOT_ARGS} || exit 1
done
done
