set -o pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv \
    -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace.log 2>&1 || exit 1
echo "trace ok"
ls $OUT/trace/*
