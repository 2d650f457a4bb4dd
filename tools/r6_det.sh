# round 6: one-stream captured step — a new batch every replay
set -o pipefail
OUT=gpurun_out/r6det
mkdir -p $OUT
export MD2_ALLOW_ONESTREAM_GRAPH=1
for ps in 0 0 1; do
  timeout -k 10 300 python -u tools/onestream_graph_check.py --pose-streams $ps --amp none --quiet 1 --vary 1 > $OUT/osv.txt 2>&1 || { tail -20 $OUT/osv.txt; exit 1; }
  echo "pose_streams $ps vary: $(grep '^quiet' $OUT/osv.txt | cut -c1-400)"
done
