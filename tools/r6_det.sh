# round 6: C5 graph replays — with the pose decoder's bf16 bias + ReLU on md2_bias_act_bwd
set -o pipefail
OUT=gpurun_out/r6det
mkdir -p $OUT
one() {  # tag, env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" python -u tools/c5_replay_diag.py --batch 32 --first graph --second graph > $OUT/$tag.txt 2>&1 || { tail -20 $OUT/$tag.txt; return 1; }
  echo "== $tag $(grep 'rel-L2 over' $OUT/$tag.txt) $(grep '^differs' $OUT/$tag.txt | head -2 | cut -c1-60 | tr '\n' ' ')"
}
timeout -k 10 300 python -u -m pytest tests/test_decoder_gpu.py -x -q -k "bias_act" --timeout 200 --timeout-method thread > $OUT/u.log 2>&1 || { tail -30 $OUT/u.log; exit 1; }
tail -1 $OUT/u.log
one ba1 A=1 && one ba2 A=1 && one ba3 A=1 && one ba4 A=1 && one ba5 A=1 && one ba6 A=1 &&
timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py -x -q -k "bf16_full_resolution" --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; tail -1 $OUT/t.log
