# round 6: bf16 stem weight gradient with the next chunk prefetched — tests, C5 trace, C5 line
set -o pipefail
OUT=gpurun_out/r6stempf
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_stem_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c5 --output-format csv \
    -- python3 bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace.log 2>&1 || exit 1
python3 tools/kstat_grep.py stem_x6 $OUT/trace/c5_kernel_stats.csv
timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --no-cpu-baseline --pmc 0 --no-eager-aten > $OUT/c5.json 2>/dev/null || exit 1
python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'], d['loss_delta_vs_oracle'])" $OUT/c5.json
