# Round-end evidence: smoke + every GPU test, bench lines for all workloads, rocprof kernel
# stats + PMC passes for the default workload and the bf16 GNN line.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_all.sh || exit $?
bash tools/gpu_profile.sh minsum-z32 ${TAG:-r01s3} || exit $?
bash tools/gpu_profile.sh gnn-z32-bf16-i10 ${TAG:-r01s3} --batch 8192 || exit $?
