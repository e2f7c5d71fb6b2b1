# Wide-H evidence on the current library: the wide tests, the h128 profile + stamped PMC summary
# (TAG), and the h128 / h192 bench lines.  usage: TAG=r06g bash tools/gpu_evidence_wide.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${TAG:-r06g}; O=$R/gpurun_out/evidence_$T; mkdir -p $O/bench
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gnn_depth_gpu.py tests/test_gnn_special_gpu.py -k "wide" > $O/pytest_wide.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
WL=gnn-z32-h128 TAG=$T bash tools/gpu_evidence_r06.sh profile || exit 1
for w in gnn-z32-h128 gnn-z32-h192; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 3 --warmup 1 --cpu-baseline-seconds 0 > $O/bench/$w.json 2> $O/bench/$w.err || { echo "bench $w rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench/$w.json')); print('$w', round(d['value']), d['roofline'].get('traffic'), d['roofline_notes'].get('wide_design_GBps'))"
done
echo "wide evidence ok"
