# Multi-rank paths rehearsed on one GPU: 2 ranks share the card, gloo for the collectives.
#   bench.py's torch.distributed.run branch (weak scaling, MAX of timings, SUM of counters) for the
#   cfg3 min-sum line, the bf16 GNN line and the cfg4 SNR sweep; the two-rank harness test.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/dist; mkdir -p $OUT
cd $R
P=29517
for W in minsum-z32 gnn-z32-bf16-i10 gnn-z32-sweep; do
  P=$((P+1))
  BENCH_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --workload $W --steps 3 --warmup 1 --batch 8192 > $OUT/$W.json 2> $OUT/$W.err || { echo "dist bench rc=$? $W"; tail -20 $OUT/$W.err; exit 1; }
  cut -c1-300 $OUT/$W.json
done
timeout -k 10 400 python -u -m pytest tests/test_sweep_dist_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; exit $rc
