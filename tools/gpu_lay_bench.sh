set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/lay; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 bench.py --workload lay-z32 --steps 10 --warmup 3 --cpu-baseline-seconds 10 > $OUT/lay.json 2> $OUT/lay.err || { echo "bench rc=$?"; tail -20 $OUT/lay.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/lay.json')); r=d['roofline']; print('lay', round(d['value']), 'cw/s', round(r['kernel_ms'],2), 'ms frac', round(r['frac'],3), 'cpu', d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload lay-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0 > $OUT/trace.log 2>&1; echo "trace rc=$?"
