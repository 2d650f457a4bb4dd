# round 6: bf16 BatchNorm reductions on eight channels per thread — tests + C5 A/B
set -o pipefail
OUT=gpurun_out/r6bnred
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 600 python -u -m pytest tests/test_trainer_gpu.py -x -q -k "bf16" --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
B="python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --pmc 0 --no-eager-aten"
for r in 1 2; do
  timeout -k 10 300 $B > $OUT/on_$r.json 2>/dev/null || exit 1
  MD2_BN_RED8=0 timeout -k 10 300 $B > $OUT/off_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'], d['loss_delta_vs_oracle'])" $OUT/on_$r.json $OUT/off_$r.json
done
