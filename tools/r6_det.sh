# round 6: one-stream captured step — find the freed block the graph still reads
set -o pipefail
OUT=gpurun_out/r6det
mkdir -p $OUT
export MD2_ALLOW_ONESTREAM_GRAPH=1
timeout -k 10 500 python -u tools/onestream_culprit.py > $OUT/culprit.txt 2>&1 || { tail -30 $OUT/culprit.txt; exit 1; }
grep -v "amdgpu.ids" $OUT/culprit.txt | tail -60
