set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u tools/conv_choices.py --batch 12 gpurun_out/r06d/conv_choices.json > gpurun_out/r06d/conv_choices.log 2>&1 || { tail -20 gpurun_out/r06d/conv_choices.log; exit 1; }
echo choices ok
ROUND=r06d MD2_CONV_CHOICES=gpurun_out/r06d/conv_choices.json bash tools/profile_round.sh
