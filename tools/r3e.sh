set -o pipefail
bash tools/ab_prof.sh r3e pk0 pk1 pk0 pk1 > gpurun_out/r3e.txt 2>&1 || exit 1
grep -v simple_timer gpurun_out/r3e.txt | grep "==\|fwdall\|ident"
