set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/lay; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py tests/test_harness_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py --workload lay-z32 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $OUT/lay.json 2> $OUT/lay.err || { echo "bench rc=$?"; tail -5 $OUT/lay.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/lay.json')); r=d['roofline']; print('lay-z32', round(d['value']), 'cw/s frac', round(r['frac'],3), 'ms', round(r['kernel_ms'],3))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload lay-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0 > $OUT/trace.log 2>&1; echo "trace rc=$?"
