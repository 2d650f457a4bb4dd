#!/bin/bash
# The same step with two pinned conv-choice tables, alternated on one box:
#   bash tools/pin_ab.sh <tag> <tableA> <tableB> [bench args]
tag=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out/$tag && export TMPDIR=/tmp
for rep in 1 2; do
  for t in A B; do
    tab=$A; [ $t = B ] && tab=$B
    MD2_CONV_CHOICES=$tab timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 \
      --no-conv-roofline "$@" > gpurun_out/$tag/$t$rep.log 2>&1 || exit 1
    echo "$t$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$tag/$t$rep.log)"
  done
done
