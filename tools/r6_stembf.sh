# round 6: C5 stem weight gradient on bf16 operands (ABI 23) — tests + C5 A/B
set -o pipefail
OUT=gpurun_out/r6s2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_stem_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py -x -q -k "bf16" --timeout 300 --timeout-method thread > $OUT/test2.log 2>&1 || { tail -30 $OUT/test2.log; exit 1; }
tail -1 $OUT/test2.log
for r in 1 2; do
  MD2_STEM_FWD_BF16=0 timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --pmc 0 --no-eager-aten > $OUT/off_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --pmc 0 --no-eager-aten > $OUT/on_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'], d['loss_delta_vs_oracle'])" $OUT/off_$r.json $OUT/on_$r.json
done
