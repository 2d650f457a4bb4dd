set -o pipefail
mkdir -p gpurun_out/r3f && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hotpath_gpu.py tests/test_abi.py > gpurun_out/r3f/tests.log 2>&1 || { tail -40 gpurun_out/r3f/tests.log; exit 1; }
tail -2 gpurun_out/r3f/tests.log
bash tools/ab_prof.sh r3f pkb0 pkb1 pkb0 pkb1 > gpurun_out/r3f/ab.txt 2>&1 || exit 1
grep -v simple_timer gpurun_out/r3f/ab.txt | grep "==\|photo_bwd\|fwdall"
