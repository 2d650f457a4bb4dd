#!/bin/bash
# hot-path parity tests + per-case error measurement (tools/parity_measure.py)
set -o pipefail
tag=${1:-par}
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/parity_measure.py gpurun_out/$tag/parity.json > gpurun_out/$tag/measure.log 2>&1 || { tail -20 gpurun_out/$tag/measure.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hotpath_gpu.py tests/test_abi.py > gpurun_out/$tag/tests.log 2>&1 || { tail -30 gpurun_out/$tag/tests.log; exit 1; }
tail -3 gpurun_out/$tag/tests.log
timeout -k 10 120 python tools/hot_bench.py --eight-bit > gpurun_out/$tag/hot_bench.log 2>&1 || exit 1
cat gpurun_out/$tag/hot_bench.log | tail -1
