set -o pipefail
mkdir -p gpurun_out/r3a && export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r3a/bench_default.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --amp bf16 --batch 32 > gpurun_out/r3a/bench_bf16_b32.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --amp bf16 --batch 32 --graph 1 > gpurun_out/r3a/bench_bf16_b32_graph.log 2>&1 || exit 1
