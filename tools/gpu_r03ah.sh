# Round 3: group-mean grid cap in listed layers (LDPC_GNN_GM_CAP) -- test, A/B on cfg5
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03ah; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_et_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'L', d.get('avg_layers'))"
}
for rep in 1 2; do
  BA="--workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1"
  run cw_cap0_$rep LDPC_GNN_GM_CAP=0
  run cw_cap64_$rep LDPC_GNN_GM_CAP=64
  run cw_cap256_$rep LDPC_GNN_GM_CAP=256
  BA="--workload gnn-z32-bf16 --steps 3 --warmup 1"
  run zero_cap0_$rep LDPC_GNN_GM_CAP=0
  run zero_cap64_$rep LDPC_GNN_GM_CAP=64
done
