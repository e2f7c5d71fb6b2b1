# Round 3: training-step knobs A/B (forward streams, backward MLP workgroup size)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03al; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']), 'ms', round(d['ms_per_step'],3))"
}
BA="--workload gnn-train-z32"
for rep in 1 2; do
  run base_$rep LDPC_GNN_STREAMS=2
  run streams1_$rep LDPC_GNN_STREAMS=1
  run mfma256_$rep LDPC_GNN_TRAIN_MFMA=2
  run projwgs2_$rep LDPC_GNN_PROJ_WGS=2
done
