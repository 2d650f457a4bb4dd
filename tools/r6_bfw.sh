set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_conv_bf16_gpu.py tests/test_conv_gpu.py -x -q -k "bf16" --timeout 250 --timeout-method thread > gpurun_out/r6/bfw_test.log 2>&1 || { tail -30 gpurun_out/r6/bfw_test.log; exit 1; }
tail -1 gpurun_out/r6/bfw_test.log
timeout -k 10 300 python -u tools/c5_conv_times.py --out gpurun_out/r6/c5_conv_times2.json > gpurun_out/r6/c5_conv_times2.log 2>&1 || { tail -20 gpurun_out/r6/c5_conv_times2.log; exit 1; }
grep -E "fwd_bf16|dgrad_bf16" gpurun_out/r6/c5_conv_times2.log | head -30
tail -1 gpurun_out/r6/c5_conv_times2.log
for r in 1 2; do
  MD2_CONV_EXCLUDE=bf16ws,bf16ws_256,bf16ws_ns,bf16ws_256_ns timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > gpurun_out/r6/bfw_off_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > gpurun_out/r6/bfw_on_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'])" gpurun_out/r6/bfw_off_$r.json gpurun_out/r6/bfw_on_$r.json
done
