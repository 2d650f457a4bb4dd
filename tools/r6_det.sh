# round 6: one-stream captured step — GPU vs host allocations between replays
set -o pipefail
OUT=gpurun_out/r6det
mkdir -p $OUT
export MD2_ALLOW_ONESTREAM_GRAPH=1
for bt in gpu host gpu host; do
  timeout -k 10 300 python -u tools/onestream_graph_check.py --pose-streams 0 --amp none --quiet 1 --between $bt > $OUT/osb.txt 2>&1 || { tail -20 $OUT/osb.txt; exit 1; }
  echo "$bt: $(grep '^quiet' $OUT/osb.txt | cut -c1-300)"
done
