set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u bench.py --amp bf16 --batch 32 --no-cpu-baseline > gpurun_out/r06/c5_line.json 2> gpurun_out/r06/c5_line.err || exit 1
echo "c5 ok"; tail -c 200 gpurun_out/r06/c5_line.json
ROUND=r06 MD2_CONV_CHOICES=profiles/r05/conv_choices.json bash tools/profile_round.sh
