# bf16 GNN: GPU tests, then the three MLP variants on cfg5 (B = 8192) and cfg2-bf16 sizes.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/bf16_ab; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gnn_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "bf16 z=|passed|failed|Error" $OUT/pytest.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for V in 0 1 2; do
  export LDPC_GNN_BF16_MLP=$V
  timeout -k 10 200 python3 bench.py --workload gnn-z32-bf16 --steps 3 --warmup 1 --batch 8192 --cpu-baseline-seconds 0 > $OUT/z32_v$V.json 2> $OUT/z32_v$V.err || { echo "bench rc=$? v$V"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/z32_v$V.json')); print('z32 v$V', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms', 'ber', d['ber'])"
done
unset LDPC_GNN_BF16_MLP
timeout -k 10 200 python3 bench.py --workload gnn-z4-bf16 --steps 5 --warmup 2 --cpu-baseline-seconds 0 > $OUT/z4.json 2> $OUT/z4.err && python3 -c "import json; d=json.load(open('$OUT/z4.json')); print('z4', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms')"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload gnn-z32-bf16 --steps 3 --warmup 1 --batch 8192 --cpu-baseline-seconds 0 > $OUT/trace.log 2>&1; echo "trace rc=$?"
head -6 $OUT/trace/run_kernel_stats.csv | cut -c1-160
