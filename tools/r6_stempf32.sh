# round 6: fp32 stem weight gradient with the next chunk prefetched (MD2_STEM_PF32) — tests + kernel A/B
set -o pipefail
OUT=gpurun_out/r6stempf32
mkdir -p $OUT
MD2_STEM_PF32=1 timeout -k 10 400 python -u -m pytest tests/test_stem_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
export TMPDIR=/tmp
for pf in 1 0; do
  MD2_STEM_PF32=$pf timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace$pf -o f32 --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-eager-aten --pmc 0 --graph 0 > $OUT/trace$pf.log 2>&1 || exit 1
  python3 tools/kstat_grep.py stem_x6_wgrad $OUT/trace$pf/f32_kernel_stats.csv
done
