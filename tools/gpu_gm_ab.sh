# A/B of the fp32 GNN group-mean kernels (LDPC_GNN_GM=0: per-group, 1: group tiles) on the
# cfg4 line (gnn-z32, 10 layers fp32), after the GNN parity tests; kernel stats for the default.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/gm_ab; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for V in ${VARIANTS:-0 1}; do
  env "${KNOB:-LDPC_GNN_GM}=$V" timeout -k 10 200 python3 bench.py --workload gnn-z32 --steps 5 --warmup 2 --batch ${BATCH:-8192} --cpu-baseline-seconds 0 > $OUT/v$V.json 2> $OUT/v$V.err || { echo "bench rc=$? v$V"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/v$V.json')); print('v$V', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload gnn-z32 --steps 3 --warmup 1 --batch ${BATCH:-8192} --cpu-baseline-seconds 0 > $OUT/trace.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cut -d, -f1-4 $OUT/trace/run_kernel_stats.csv | head -6
