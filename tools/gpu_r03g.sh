# Round 3 re-entry: smoke, full -m gpu suite on HEAD, then the headline and GNN bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 200 python -u -m pytest tests/test_train_gpu.py -q -k deep --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_ds.log 2>&1 || { tail -30 $O/pytest_ds.log; exit 1; }
tail -2 $O/pytest_ds.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'frac', round(r['frac'],3), 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'), 'avg_layers', d.get('avg_layers'))"
}
run minsum-z32 --steps 20 --warmup 3 --cpu-baseline-seconds 0
run gnn-z32-bf16 --workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32-bf16-i10 --workload gnn-z32-bf16-i10 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32 --workload gnn-z32 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-train-z32 --workload gnn-train-z32 --steps 10 --warmup 2 --cpu-baseline-seconds 0
run minsum-z32-stream --workload minsum-z32-stream --steps 10 --warmup 2 --cpu-baseline-seconds 0
