# Round-end evidence: the whole -m gpu suite, then one bench line per workload (the default cfg3
# line with its CPU baseline).  Outputs under gpurun_out/final/ (copy into profiles/ to keep).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/final; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $O/minsum_z32.json || exit $?
B="timeout -k 10 300 python bench.py --cpu-baseline-seconds 0"
for w in ${WORKLOADS:-bp-z32 minsum-z32-stream minsum-z384 gnn-z32 gnn-z32-bf16-i10 gnn-z32-bf16 gnn-z32-sweep gnn-train-z32 lay-z32 hybrid-minsum-z32 hybrid-gnn-z32}; do
  $B --workload $w > $O/${w//-/_}.json || { echo "bench $w rc=$?"; exit 1; }
done
$B --early-stop batch --snr 6 --iterations 50 > $O/minsum_z32_es_batch_6db.json && \
$B --early-stop frame --snr 6 --iterations 50 > $O/minsum_z32_es_frame_6db.json || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', round(d['value']), 'cw/s', round(d['ms_per_step'],3), 'ms', r['bound'], None if r['frac'] is None else round(r['frac'],3))"; done
