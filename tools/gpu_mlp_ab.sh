# A/B of the fp32 MFMA MLP variants (LDPC_GNN_MLP_THREADS 256/512 x LDPC_GNN_MLP_PF 0/1) on the
# cfg4 line (gnn-z32, 10 layers fp32, B = 8192), after the fp32 GNN parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/mlp_ab; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for V in ${VARIANTS:-512:1 512:0 256:1 256:0}; do
  T=${V%:*}; P=${V#*:}; n=t${T}_pf$P
  LDPC_GNN_MLP_THREADS=$T LDPC_GNN_MLP_PF=$P timeout -k 10 200 python3 bench.py --workload gnn-z32 --steps 5 --warmup 2 --batch ${BATCH:-8192} --cpu-baseline-seconds 0 > $OUT/$n.json 2> $OUT/$n.err || { echo "bench rc=$? $n"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],3))"
done
