# Round 3: training backward's projection recompute on a side stream (LDPC_GNN_TRAIN_OVERLAP) -- tests, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03aj; mkdir -p $O
LDPC_GNN_TRAIN_OVERLAP=1 timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'ms', round(d['ms_per_step'],3), 'kern_ms', round(r['kernel_ms'],3))"
}
BA="--workload gnn-train-z32"
for rep in 1 2 3; do
  run ovl0_$rep LDPC_GNN_TRAIN_OVERLAP=0
  run ovl1_$rep LDPC_GNN_TRAIN_OVERLAP=1
done
