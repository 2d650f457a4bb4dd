set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -k "warp_specialised" --timeout 250 --timeout-method thread > gpurun_out/r6/wws_test2.log 2>&1 || { tail -30 gpurun_out/r6/wws_test2.log; exit 1; }
tail -1 gpurun_out/r6/wws_test2.log
timeout -k 10 300 python -u tools/wgrad_bench.py > gpurun_out/r6/wws_bench2.log 2>&1 || { tail -20 gpurun_out/r6/wws_bench2.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r6/wws_bench2.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if 'x6ws' in d: print(d['name'], d['x6'], d['x6ws'])
"
