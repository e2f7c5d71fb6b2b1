# Round-5 refresh after the staged check rows, the f16 projection and the LDS output kernel: profiles +
# stamped PMC summaries of the fp32 GNN forward and the training step, then the bench lines whose
# kernels changed.  usage: TAG=r05z3 bash tools/gpu_evidence_z.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${TAG:-r05z3}
TAG=$T bash tools/gpu_evidence_y.sh profile || exit 1
O=$R/gpurun_out/evidence_$T/bench; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), d['unit'], 'frac', None if r['frac'] is None else round(r['frac'],3), 'traffic', r.get('traffic'), 'kern_ms', round(r['kernel_ms'],2))"
}
run gnn-z32 --workload gnn-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 10
run gnn-train-z32 --workload gnn-train-z32 --steps 5 --warmup 2 --cpu-baseline-seconds 10
run gnn-z32-bf16 --workload gnn-z32-bf16 --steps 3 --warmup 1 --cpu-baseline-seconds 10
run hybrid-gnn-z32 --workload hybrid-gnn-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z4 --workload gnn-z4 --steps 10 --warmup 3 --cpu-baseline-seconds 10
