# Round 3: msg_out variable-major (default) vs message order on cfg5 -- test, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03ac; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_et_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'L', d.get('avg_layers'))"
}
BA="--workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1"
for rep in 1 2; do
  run vm1_$rep LDPC_GNN_MSGOUT_VM=1
  run vm0_$rep LDPC_GNN_MSGOUT_VM=0
done
