# Batch-size sweep of one workload + a kernel trace at two sizes (per-kernel durations).
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/bsweep; mkdir -p $OUT
cd $R
W=${W:-gnn-z32-bf16-i10}
for B in ${BATCHES:-4096 8192 16384 32768}; do
  timeout -k 10 300 python3 bench.py --workload $W --steps ${STEPS:-6} --warmup ${WARM:-4} --batch $B --cpu-baseline-seconds 0 > $OUT/b$B.json 2> $OUT/b$B.err || { echo "bench rc=$? B=$B"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$B.json')); print('B=$B', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms', round(d['roofline']['kernel_ms']*1e3/$B,2), 'us/frame')"
done
cd /tmp && export TMPDIR=/tmp
for B in ${TRACE_BATCHES:-8192 32768}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_b$B -o run -- python3 $R/bench.py --workload $W --steps 3 --warmup 3 --batch $B --cpu-baseline-seconds 0 > $OUT/trace_b$B.log 2>&1 || { echo "trace rc=$?"; exit 1; }
done
echo done
