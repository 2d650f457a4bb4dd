#!/bin/bash
# A/B of the HIP runtime's graph-execution knobs on the captured bf16 B=32 step.
set -o pipefail
mkdir -p gpurun_out/gsweep && export TMPDIR=/tmp
run() { tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --amp bf16 --batch 32 --graph 1 > gpurun_out/gsweep/$tag.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/gsweep/$tag.log | sed "s/^/$tag /"
}
run base A=1
run q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
run q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run pc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run bs64 DEBUG_HIP_GRAPH_BATCH_SIZE=64
run bs1024 DEBUG_HIP_GRAPH_BATCH_SIZE=1024
