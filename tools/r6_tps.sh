# round 6: three taps per barrier in the bf16 patch kernel — tests, C5 table, C5 A/B
set -o pipefail
OUT=gpurun_out/r6t
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_bf16_gpu.py -x -q --timeout 250 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 300 python -u tools/c5_conv_times.py --out $OUT/c5_conv_times.json > $OUT/c5_conv_times.log 2>&1 || { tail -20 $OUT/c5_conv_times.log; exit 1; }
tail -1 $OUT/c5_conv_times.log
for r in 1 2; do
  MD2_LIB=ab7/old/libmd2hot.so timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > $OUT/old_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > $OUT/new_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'])" $OUT/old_$r.json $OUT/new_$r.json
done
