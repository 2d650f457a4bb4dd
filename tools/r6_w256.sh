set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -k "warp_specialised or 256_wide" --timeout 250 --timeout-method thread > gpurun_out/r6/w256_test.log 2>&1 || { tail -30 gpurun_out/r6/w256_test.log; exit 1; }
tail -1 gpurun_out/r6/w256_test.log
timeout -k 10 300 python -u tools/wgrad_bench.py > gpurun_out/r6/w256_bench.log 2>&1 || { tail -20 gpurun_out/r6/w256_bench.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r6/w256_bench.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if 'x6ws' in d: print(d['name'], d['x6'], d['x6ws'], d['x6ws_256'], d.get('x6pw'), d['miopen'], d['err_x6'], d['err_x6ws_256'])
"
for r in 1 2; do
  MD2_CONV_EXCLUDE=x6ws_256 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > gpurun_out/r6/w256_off_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --pmc 0 --no-eager-aten > gpurun_out/r6/w256_on_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys
for f in sys.argv[1:]: d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'])" gpurun_out/r6/w256_off_$r.json gpurun_out/r6/w256_on_$r.json
done
