# Multi-rank bench path rehearsed on one GPU: 2 ranks share the card, gloo for the collectives.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/dist; mkdir -p $OUT
cd $R
for W in minsum-z32 gnn-z32-bf16-i10; do
  BENCH_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload $W --steps 3 --warmup 1 --batch 8192 > $OUT/$W.json 2> $OUT/$W.err || { echo "dist bench rc=$? $W"; tail -20 $OUT/$W.err; exit 1; }
  cat $OUT/$W.json | cut -c1-400
done
