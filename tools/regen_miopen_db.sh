#!/bin/bash
# Regenerate the shipped MIOpen find-db / perf-db / kernel cache (monodepth2_amd/miopen_db)
# on a GPU box: an exhaustive MIOpen find (MIOPEN_FIND_MODE=NORMAL) over every
# convolution shape of the bench configurations, into a fresh directory.  Run from the
# repo root on the box (gpurun), then copy gpurun_out/miopen_db_new/* over
# monodepth2_amd/miopen_db/ in the source tree.  Takes a few minutes per configuration.
set -o pipefail
OUT=gpurun_out/miopen_db_new
rm -rf $OUT && mkdir -p $OUT
export MIOPEN_FIND_MODE=NORMAL MIOPEN_USER_DB_PATH=$OUT MIOPEN_CUSTOM_CACHE_DIR=$OUT TMPDIR=/tmp
for cfg in "" "--amp bf16 --batch 32" "--amp bf16" "--stereo" "--num_layers 50 --height 320 --width 1024 --batch 8"; do
  echo "== $cfg"
  timeout -k 10 900 python bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-parity --pmc 0 --no-conv-roofline \
      --miopen-find normal $cfg > $OUT/log_$(echo $cfg | tr ' -' '__').txt 2>&1 || exit 1
done
ls -la $OUT
