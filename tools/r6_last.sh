# round 6: last tree — stem / conv / trainer GPU tests and smoke
set -o pipefail
OUT=gpurun_out/r6last
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_stem_gpu.py tests/test_conv_gpu.py tests/test_conv_bf16_gpu.py tests/test_trainer_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
