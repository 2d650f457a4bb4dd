#!/bin/bash
# HBM bytes per launch of every hand-written kernel of the step (FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes over the bench command); summarise with
# tools/kernel_hbm_table.py.  Output: gpurun_out/$ROUND/hbm{0,1}/
set -o pipefail
ROUND=${ROUND:-r02}
OUT=gpurun_out/$ROUND
mkdir -p $OUT
export TMPDIR=/tmp
RE="photo_|pack_src8|disp_grad|smooth_fwd|grad_T|finalize|pad_fwd|pad_bwd|bias_grad|pose_|bn_|head_|adam|maxpool|encoder_input|bias_act|conv_x6|conv_wsplit|conv_reduce"
i=0
for p in "FETCH_SIZE" "WRITE_SIZE"; do
    timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "$RE" \
        -d $OUT/hbm$i -o pmc --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity \
        > $OUT/hbm$i.log 2>&1 || exit 1
    echo "hbm pass $i ($p) ok"
    i=$((i+1))
done
