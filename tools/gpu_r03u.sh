# Round 3: bf16 MLP occupancy variants (LDPC_GNN_BF16_MLP 1 = 2 waves + prefetch, 0 = 3 waves, 4 = 3 waves + prefetch, 5 = 4 waves)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03u; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3))"
}
BA="--workload gnn-z32-bf16-i10 --steps 3 --warmup 1"
for v in 1 0 4 5 3; do run v$v LDPC_GNN_BF16_MLP=$v; done
