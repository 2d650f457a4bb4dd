# round 6: factorised projection (M = P inv_K) + dL/dP accumulation — hot-path A/B and parity
set -o pipefail
OUT=gpurun_out/r6p
mkdir -p $OUT
hb() { timeout -k 5 120 python tools/hot_bench.py --eight-bit --src8 "$@"; }
for rep in 1 2 3; do
  MD2_LIB=ab6/old/libmd2hot.so hb > $OUT/old_$rep.json || exit 1
  MD2_LIB=ab6/new/libmd2hot.so hb > $OUT/new_$rep.json || exit 1
done
for f in $OUT/*.json; do echo "$f $(cat $f)"; done
timeout -k 10 600 python -u -m pytest tests/test_hotpath_gpu.py tests/test_parity_floor_gpu.py tests/test_trainer_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
