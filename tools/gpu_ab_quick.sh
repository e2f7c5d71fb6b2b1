# Quick A/B of the bf16 GNN MLP variants on the 10-layer cfg4-shape line (B = 8192).
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/ab_quick; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for V in ${VARIANTS:-0 1}; do
  export LDPC_GNN_BF16_MLP=$V
  timeout -k 10 200 python3 bench.py --workload gnn-z32-bf16-i10 --steps ${STEPS:-10} --warmup ${WARM:-5} --batch ${BATCH:-8192} --cpu-baseline-seconds 0 > $OUT/v$V.json 2> $OUT/v$V.err || { echo "bench rc=$? v$V"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/v$V.json')); print('v$V', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],3))"
done
