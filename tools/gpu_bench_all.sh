# Bench lines for every workload into gpurun_out/bench_all (one JSON line each).
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/bench_all; mkdir -p $OUT
cd $R
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $OUT/$n.json 2> $OUT/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); r=d['roofline']; c=d['cpu_baseline'] or {}; print('$n', round(d['value']), d['unit'], 'frac', None if r['frac'] is None else round(r['frac'],3), 'kern_ms', round(r['kernel_ms'],2), 'cpu', c.get('value'))"
}
run minsum-z32 --steps 20 --warmup 3
run bp-z4 --workload bp-z4 --batch 65536 --steps 10 --warmup 3 --cpu-baseline-seconds 5
run bp-z32 --workload bp-z32 --steps 10 --warmup 3 --cpu-baseline-seconds 5
run gnn-z4 --workload gnn-z4 --steps 10 --warmup 3 --cpu-baseline-seconds 10
run gnn-z4-bf16 --workload gnn-z4-bf16 --steps 10 --warmup 3 --cpu-baseline-seconds 0
run gnn-z32 --workload gnn-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 10
run gnn-z32-h128 --workload gnn-z32-h128 --steps 3 --warmup 1 --cpu-baseline-seconds 10
run gnn-z32-h192 --workload gnn-z32-h192 --steps 2 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32-codewords --workload gnn-z32 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32-bf16 --workload gnn-z32-bf16 --steps 3 --warmup 1 --cpu-baseline-seconds 10
run gnn-z32-bf16-codewords --workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32-bf16-noet --workload gnn-z32-bf16 --early-termination off --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32-bf16-codewords-noet --workload gnn-z32-bf16 --data codewords --early-termination off --steps 3 --warmup 1 --cpu-baseline-seconds 0
run gnn-z32-bf16-i10 --workload gnn-z32-bf16-i10 --steps 3 --warmup 1 --cpu-baseline-seconds 10
run gnn-train-z32 --workload gnn-train-z32 --steps 5 --warmup 2 --cpu-baseline-seconds 10
run gnn-train-z4 --workload gnn-train-z4 --steps 5 --warmup 2 --cpu-baseline-seconds 10
run lay-z32 --workload lay-z32 --steps 10 --warmup 3 --cpu-baseline-seconds 10
run gnn-z32-sweep --workload gnn-z32-sweep --steps 1 --warmup 1 --cpu-baseline-seconds 0
run minsum-z32-stream --workload minsum-z32-stream --steps 10 --warmup 2 --cpu-baseline-seconds 5
run minsum-z384 --workload minsum-z384 --steps 5 --warmup 2 --cpu-baseline-seconds 0
run hybrid-minsum-z32 --workload hybrid-minsum-z32 --steps 10 --warmup 2 --cpu-baseline-seconds 0
run hybrid-gnn-z32 --workload hybrid-gnn-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0
run minsum-z32-es-batch-6db --early-stop batch --iterations 50 --snr 6 --steps 20 --warmup 3 --cpu-baseline-seconds 0
run minsum-z32-es-frame-6db --early-stop frame --iterations 50 --snr 6 --steps 20 --warmup 3 --cpu-baseline-seconds 0
