# cfg5 (bf16, 15 layers) with and without early termination: bench lines + kernel traces.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/et_prof; mkdir -p $OUT
cd $R
for ET in ${BENCH_ET:-}; do
  timeout -k 10 300 python3 bench.py --workload gnn-z32-bf16 --early-termination $ET --steps 5 --warmup 3 --batch 8192 --cpu-baseline-seconds 0 > $OUT/$ET.json 2> $OUT/$ET.err || { echo "bench rc=$? $ET"; tail -20 $OUT/$ET.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$ET.json')); print('$ET', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms', 'avg_layers', d['avg_layers'])"
done
cd /tmp && export TMPDIR=/tmp
for ET in on off; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$ET -o run -- python3 $R/bench.py --workload gnn-z32-bf16 --early-termination $ET --steps 2 --warmup 1 --batch 8192 --cpu-baseline-seconds 0 > $OUT/trace_$ET.log 2>&1 || { echo "trace rc=$? $ET"; exit 1; }
done
