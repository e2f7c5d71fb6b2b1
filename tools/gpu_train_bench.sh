set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/train_bench; mkdir -p $OUT
cd $R
for W in gnn-train-z4 gnn-train-z32; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-baseline-seconds 10 > $OUT/$W.json 2> $OUT/$W.err || { echo "bench rc=$? $W"; tail -20 $OUT/$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$W.json')); r=d['roofline']; print('$W', round(d['value']), d['unit'], 'ms', round(d['ms_per_step'],2), 'frac', round(r['frac'],3), 'cpu', d['cpu_baseline']['value'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload gnn-train-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0 > $OUT/trace.log 2>&1; echo "trace rc=$?"
