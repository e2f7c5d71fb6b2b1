set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/et; mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gnn_et_gpu.py tests/test_gnn_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for W in gnn-z32-bf16 gnn-z32-bf16-i10; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 5 --warmup 3 --batch 8192 --cpu-baseline-seconds 0 > $OUT/$W.json 2> $OUT/$W.err || { echo "bench rc=$? $W"; tail -20 $OUT/$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$W.json')); print('$W', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms', 'avg_layers', d['avg_layers'])"
done
