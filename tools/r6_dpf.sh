# round 6: direct 16-channel forward with the next tile's patch prefetched — tests, C5 trace, bench lines
set -o pipefail
OUT=gpurun_out/r6dpf
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_conv_bf16_gpu.py -x -q -k "direct" --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c5 --output-format csv \
    -- python3 bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace32 -o f32 --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace32.log 2>&1 || exit 1
python3 tools/kstat_grep.py conv3_x6 $OUT/trace/c5_kernel_stats.csv $OUT/trace32/f32_kernel_stats.csv
B="python -u bench.py --no-cpu-baseline --pmc 0 --no-eager-aten"
timeout -k 10 300 $B --amp bf16 --batch 32 > $OUT/c5.json 2>/dev/null || exit 1
timeout -k 10 300 $B > $OUT/f32.json 2>/dev/null || exit 1
python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'], d['loss_delta_vs_oracle'])" $OUT/c5.json $OUT/f32.json
