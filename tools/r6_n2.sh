# N>1 bench path rehearsed on one GPU: two ranks over gloo (DDP eager), and the captured
# step's refusal on gloo
set -o pipefail
OUT=gpurun_out/r6n2
mkdir -p $OUT
export MD2_DIST_BACKEND=gloo MD2_DEVICE_INDEX=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/n2.json 2> $OUT/n2.err || { tail -30 $OUT/n2.err; exit 1; }
tail -c 400 $OUT/n2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --graph 1 > $OUT/n2g.json 2> $OUT/n2g.err; echo "graph-on-gloo exit $?"; grep -m2 -i "refus\|rccl\|nccl" $OUT/n2g.err
