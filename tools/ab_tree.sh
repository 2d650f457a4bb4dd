#!/bin/bash
# Same-box A/B of the bench: variants/headtree (a git worktree of an earlier commit,
# built in place) vs this tree, alternating.  [BENCH_ARGS=...] tools/ab_tree.sh [rounds]
set -o pipefail
n=${1:-2}
mkdir -p gpurun_out
for i in $(seq $n); do
  for t in variants/headtree .; do
    (cd $t && timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity $BENCH_ARGS) \
        > gpurun_out/abt.log 2>&1 || exit 1
    echo "$t: $(grep -o 'timed: [0-9.]* ms/step' gpurun_out/abt.log) $(grep -o 'host enqueue time: [0-9.]* ms/step' gpurun_out/abt.log)"
  done
done
