set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gnn_gpu.py tests/test_gnn_depth_gpu.py tests/test_gnn_et_gpu.py tests/test_checkpoints_gpu.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sub.log; [ $rc -eq 0 ] || exit $rc
TAG=i10 bash tools/gpu_ab.sh "gnn_r04base" "" --workload gnn-z32-bf16-i10 --steps 3 --warmup 1 || exit 1
TAG=cfg5cw bash tools/gpu_ab.sh "gnn_r04base" "" --workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1
