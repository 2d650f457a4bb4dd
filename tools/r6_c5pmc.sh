# PMC of config C5's bf16 convolution kernels: MFMA busy vs LDS-array activity
set -o pipefail
OUT=gpurun_out/r6c5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 3 --warmup 3 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten --graph 0 > $OUT/warm.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "conv_x6|conv3_x6|stem_x6|conv_reduce" -d $OUT/pmc -o pmc --output-format csv \
    -- python3 bench.py --amp bf16 --batch 32 --steps 3 --warmup 3 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten --graph 0 > $OUT/pmc.log 2>&1 || exit 1
echo pmc ok
ls $OUT/pmc/*
