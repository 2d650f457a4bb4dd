#!/bin/bash
# Collect the round's rocprofv3 evidence on a GPU box (run from the repo root):
#   kernel trace + stats of the default bench command, then separate --pmc passes
#   (FETCH_SIZE / WRITE_SIZE / SQ issue counters / L2 hit / texture address+data
#   unit busy) on the hot-path kernels.
# Output: gpurun_out/$ROUND/...; summarise with tools/make_profile_summary.py.
set -o pipefail
ROUND=${ROUND:-r04}
# MD2_CONV_CHOICES=<table> (tools/conv_choices.py) pins the convolution choices: no
# autotune timing runs inside the profiled steps
OUT=gpurun_out/$ROUND
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv \
    -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace.log 2>&1 || exit 1
echo "trace ok"
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "photo_|pack_src8|disp_grad|smooth_fwd|grad_T|finalize_fwd|conv_x6|conv3_x6|conv_wsplit|stem_x6|col2im|bn_" \
        -d $OUT/pmc$i -o pmc --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 \
        > $OUT/pmc$i.log 2>&1 || exit 1
    echo "pmc pass $i ($p) ok"
    i=$((i+1))
done
