# BP checks (fixtures, oracle, variants) and the BP bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/bp; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_flood_gpu.py tests/test_harness_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for W in bp-z32 bp-z4; do
  timeout -k 10 200 python3 bench.py --workload $W --batch 65536 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $OUT/$W.json 2> $OUT/$W.err || { echo "bench rc=$? $W"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$W.json')); print('$W', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms ber', d.get('ber'), 'fer', d.get('fer'))"
done
