# A/B of the degree-1 var-group skip (LDPC_GNN_BF16_D1) on the bf16 GNN lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/ab_d1; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py tests/test_gnn_et_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep "bf16 z=" $OUT/pytest.log || true
for W in gnn-z32-bf16-i10 gnn-z4-bf16; do
for V in 0 1; do
  export LDPC_GNN_BF16_D1=$V
  timeout -k 10 200 python3 bench.py --workload $W --steps ${STEPS:-10} --warmup ${WARM:-5} --cpu-baseline-seconds 0 > $OUT/$W-d$V.json 2> $OUT/$W-d$V.err || { echo "bench rc=$? $W d$V"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$W-d$V.json')); print('$W d$V', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],3), 'ms frac', round(d['roofline']['frac'],3))"
done
done
