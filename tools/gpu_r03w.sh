# Round 3: bf16 MLP with the group rows both GEMM1 first (LDPC_GNN_BF16_MLP=8) vs default (1)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_et_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'L', d.get('avg_layers'))"
}
for rep in 1 2; do
  BA="--workload gnn-z32-bf16-i10 --steps 3 --warmup 1"
  run i10_v1_$rep LDPC_GNN_BF16_MLP=1
  run i10_v8_$rep LDPC_GNN_BF16_MLP=8
done
BA="--workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1"
run cfg5_v1 LDPC_GNN_BF16_MLP=1
run cfg5_v8 LDPC_GNN_BF16_MLP=8
