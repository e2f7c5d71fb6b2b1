set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/flood; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_flood_gpu.py tests/test_channel_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $OUT/ms.json 2> $OUT/ms.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/ms.json')); r=d['roofline']; print('minsum-z32', round(d['value']), 'cw/s', round(r['kernel_ms'],3), 'ms')"
timeout -k 10 300 python3 bench.py --workload bp-z4 --batch 65536 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $OUT/bp.json 2> $OUT/bp.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/bp.json')); r=d['roofline']; print('bp-z4', round(d['value']), 'cw/s', round(r['kernel_ms'],3), 'ms')"
