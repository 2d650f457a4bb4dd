#!/bin/bash
# The same training step under two environment settings, alternated on one box with the
# pinned conv-choice table (so the autotune's timing noise is not part of the A/B):
#   bash tools/env_ab.sh <tag> "<VAR=v ...>" "<VAR=v ...>" [reps] [bench args]
tag=$1; A=$2; B=$3; reps=${4:-3}; shift 4
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
export MD2_CONV_CHOICES=${MD2_CONV_CHOICES:-monodepth2_amd/conv_choices.json}
for rep in $(seq 1 $reps); do
  for t in A B; do
    e=$A; [ $t = B ] && e=$B
    env $e timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 \
      --no-conv-roofline "$@" > gpurun_out/$tag/$t$rep.log 2>&1 || exit 1
    echo "$t$rep [$e] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$tag/$t$rep.log)"
  done
done
