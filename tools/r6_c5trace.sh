# kernel trace of config C5's eager step (bf16 autocast, B=32)
set -o pipefail
OUT=gpurun_out/r6c5t6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c5 --output-format csv \
    -- python3 bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace.log 2>&1 || exit 1
echo trace ok
