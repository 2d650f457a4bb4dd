set -o pipefail
bash tools/step_trace.sh r3c conv_reduce bn_ SubTensor conv_wsplit > /dev/null || exit 1
bash tools/ab_prof.sh r3c_rp rp16 rp10 rp13 rp19 rp16 > gpurun_out/r3c_rp.txt 2>&1 || exit 1
cat gpurun_out/r3c_rp.txt
