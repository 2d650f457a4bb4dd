# round 6: warp-specialised x6 weight gradient — bitwise test, per-shape timings, step A/B
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -k "warp_specialised or split_bf16" --timeout 250 --timeout-method thread > gpurun_out/r6/wws_test.log 2>&1 || { tail -30 gpurun_out/r6/wws_test.log; exit 1; }
tail -2 gpurun_out/r6/wws_test.log
timeout -k 10 300 python -u tools/wgrad_bench.py > gpurun_out/r6/wws_bench.log 2>&1 || { tail -20 gpurun_out/r6/wws_bench.log; exit 1; }
cat gpurun_out/r6/wws_bench.log | grep name
for r in 1 2; do
  MD2_CONV_EXCLUDE=x6ws timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > gpurun_out/r6/wws_off_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > gpurun_out/r6/wws_on_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'])" gpurun_out/r6/wws_off_$r.json gpurun_out/r6/wws_on_$r.json
done
