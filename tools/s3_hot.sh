#!/bin/bash
# Session-3 hot-path A/B (small-kernel unrolls) + hot-path GPU tests at this tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
HOT_ARGS="" bash tools/ab_hot.sh hbase hsm hsm2 hsm3 > gpurun_out/s3/ab_hot2.log 2>&1 || exit 1
echo abhot ok
timeout -k 10 400 python -u -m pytest tests/test_hotpath_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/tests_hot.log 2>&1 || exit 1
echo tests ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/s3hot -o hot --output-format csv -- python3 tools/hot_bench.py --iters 40 > gpurun_out/s3/hot_prof.log 2>&1 || exit 1
echo prof ok
