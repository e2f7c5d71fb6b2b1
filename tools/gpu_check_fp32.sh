# All GPU tests, then the fp32 GNN, BP Z=32 and training bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/check_fp32; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $OUT/$n.json 2> $OUT/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); r=d['roofline']; c=d['cpu_baseline'] or {}; print('$n', round(d['value']), d['unit'], 'frac', round(r['frac'],3), 'kern_ms', round(r['kernel_ms'],2), 'cpu', c.get('value'))"
}
run bp-z32 --workload bp-z32 --steps 10 --warmup 3 --cpu-baseline-seconds 5
run gnn-z32 --workload gnn-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z4 --workload gnn-z4 --steps 10 --warmup 3 --cpu-baseline-seconds 0
run gnn-train-z32 --workload gnn-train-z32 --steps 5 --warmup 2 --cpu-baseline-seconds 0
