# Flood decoder check after a kernel change: flood/harness tests, then bench lines (cfg3 default,
# early-stop variants at 6 dB and 2 dB, BP Z=32).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fl
timeout -k 10 600 python -u -m pytest tests/test_flood_gpu.py tests/test_harness_gpu.py tests/test_channel_gpu.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/fl/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/fl/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 120 python bench.py --cpu-baseline-seconds 0"
$B > gpurun_out/fl/minsum.json && \
$B --early-stop batch --snr 6 --iterations 50 > gpurun_out/fl/es_batch_6db.json && \
$B --early-stop frame --snr 6 --iterations 50 > gpurun_out/fl/es_frame_6db.json && \
$B --early-stop batch --snr 2 --iterations 50 > gpurun_out/fl/es_batch_2db.json && \
$B --early-stop frame --snr 2 --iterations 50 > gpurun_out/fl/es_frame_2db.json && \
$B --workload bp-z32 > gpurun_out/fl/bp.json
rc=$?
for f in gpurun_out/fl/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']), d['ms_per_step'], d.get('avg_iterations'), d['ber'])"; done
exit $rc
