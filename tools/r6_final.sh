# round-6 final tree: GPU suite, smoke, default bench line, C5 / C3 / C4 lines
set -o pipefail
OUT=gpurun_out/r6f5
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench_line.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --no-cpu-baseline > $OUT/bench_line_c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 300 python -u bench.py --stereo --no-cpu-baseline > $OUT/bench_line_c3.json 2> $OUT/c3.err || exit 1
timeout -k 10 400 python -u bench.py --num_layers 50 --height 320 --width 1024 --batch 8 --no-cpu-baseline > $OUT/bench_line_c4.json 2> $OUT/c4.err || exit 1
for f in $OUT/bench_line*.json; do python3 -c "import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('loss_delta_vs_oracle'), d['roofline'].get('frac') if d.get('roofline') else None)" $f; done
