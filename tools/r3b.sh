set -o pipefail
mkdir -p gpurun_out/r3b && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "plane_bank or presplit" tests/test_trainer_gpu.py::test_plane_bank_step_matches_per_call_splits tests/test_trainer_gpu.py::test_hip_graph_replay_matches_eager_step > gpurun_out/r3b/tests.log 2>&1 || { tail -40 gpurun_out/r3b/tests.log; exit 1; }
tail -3 gpurun_out/r3b/tests.log
for v in 0 1 0 1; do
MD2_PLANE_BANK=$v timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity --pmc 0 > gpurun_out/r3b/bench_$v.log 2>&1 || exit 1
python -c "import json,sys; d=json.loads(open('gpurun_out/r3b/bench_$v.log').read().strip().splitlines()[-1]); print('bank=$v', d['ms_per_step'], d['value'])"
done
