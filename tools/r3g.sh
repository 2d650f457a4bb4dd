set -o pipefail
mkdir -p gpurun_out/r3g && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3g/gputests.log 2>&1 || { tail -40 gpurun_out/r3g/gputests.log; exit 1; }
tail -2 gpurun_out/r3g/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g/smoke.log 2>&1 || { tail -5 gpurun_out/r3g/smoke.log; exit 1; }
tail -1 gpurun_out/r3g/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3g/bench.log 2>&1 || { tail -20 gpurun_out/r3g/bench.log; exit 1; }
tail -1 gpurun_out/r3g/bench.log | cut -c1-300
bash tools/hot_prof.sh r3g_hp
