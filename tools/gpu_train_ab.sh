# Training backward: parity (both MFMA variants) + A/B of the MLP backward kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/train_ab; mkdir -p $OUT
cd $R
for V in 1; do
  LDPC_GNN_TRAIN_MFMA=$V timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py tests/test_harness_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_v$V.log 2>&1 || { echo "pytest v$V failed"; tail -30 $OUT/pytest_v$V.log; exit 1; }
  tail -1 $OUT/pytest_v$V.log
done
for V in 1; do
  LDPC_GNN_TRAIN_MFMA=$V timeout -k 10 300 python3 bench.py --workload gnn-train-z32 --steps 5 --warmup 2 --cpu-baseline-seconds 0 > $OUT/z32_v$V.json 2> $OUT/z32_v$V.err || { echo "bench rc=$? v$V"; tail -5 $OUT/z32_v$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/z32_v$V.json')); print('v$V', round(d['value']), 'cw/s', round(d['ms_per_step'],2), 'ms/step')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload gnn-train-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0 > $OUT/trace.log 2>&1; echo "trace rc=$?"
