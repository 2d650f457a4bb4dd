set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u tools/c5_conv_times.py --amp none --batch 12 --out gpurun_out/r6/fp32_conv_times.json > gpurun_out/r6/fp32_conv_times.log 2>&1 || { tail -20 gpurun_out/r6/fp32_conv_times.log; exit 1; }
head -40 gpurun_out/r6/fp32_conv_times.log
tail -1 gpurun_out/r6/fp32_conv_times.log
