#!/bin/bash
# Session-3 profiling call at the session's tree: per-step kernel breakdown of the eager
# step, the round's rocprofv3 trace + PMC passes (tools/profile_round.sh), default bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
bash tools/step_trace.sh s3trace3 > gpurun_out/s3/step_trace.log 2>&1 || exit 1
echo steptrace ok
ROUND=r03s3 bash tools/profile_round.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/s3/bench_final.log 2>&1 || exit 1
echo bench ok
