#!/bin/bash
# Session-3 profiling call: the round's rocprofv3 trace + PMC passes (tools/profile_round.sh)
# at the session's final tree, then the default bench line.
set -o pipefail
export TMPDIR=/tmp
ROUND=r03s3 bash tools/profile_round.sh || exit 1
mkdir -p gpurun_out/s3
timeout -k 10 300 python bench.py > gpurun_out/s3/bench_final.log 2>&1 || exit 1
echo bench ok
