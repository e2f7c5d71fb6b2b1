set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r01i
timeout -k 10 600 python -m pytest $R/tests/test_gnn_gpu.py -m gpu -q -s -p no:cacheprovider > $R/gpurun_out/r01i/pytest_gnn.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "bf16 z=|passed|failed" $R/gpurun_out/r01i/pytest_gnn.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash $R/tools/gpu_bench.sh r01i gnn-z32-bf16 --steps 3 --warmup 1 --batch 8192 --cpu-baseline-seconds 0 || exit $?
bash $R/tools/gpu_bench.sh r01i gnn-z32 --steps 3 --warmup 1 --batch 8192 --cpu-baseline-seconds 0
