#!/bin/bash
# PMC passes over tools/hot_bench.py for one variant build (photo kernels only).
#   tools/pmc_hot.sh VARIANT TAG "COUNTERS" ["COUNTERS" ...]
set -o pipefail
v=$1; tag=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$tag
i=0
for p in "$@"; do
  MD2_LIB=variants/$v/libmd2hot.so timeout -s KILL 90 rocprofv3 --pmc $p --kernel-include-regex "photo_" \
      -d gpurun_out/pmc_$tag/p$i -o pmc --output-format csv -- python3 tools/hot_bench.py --iters 10 \
      > gpurun_out/pmc_$tag/p$i.log 2>&1 || exit 1
  i=$((i+1))
done
