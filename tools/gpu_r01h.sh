set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r01h
timeout -k 10 600 python -m pytest $R/tests/test_gnn_gpu.py -m gpu -q -s -p no:cacheprovider > $R/gpurun_out/r01h/pytest_gnn.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "bf16 z=|passed|failed" $R/gpurun_out/r01h/pytest_gnn.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash $R/tools/gpu_ab.sh r01h_fp32 gnn-z32 "LDPC_GNN_MLP_THREADS=256" "LDPC_GNN_MLP_THREADS=512" || exit $?
bash $R/tools/gpu_multi.sh r01h "gnn-z32-bf16 --steps 3 --warmup 1 --batch 8192 --cpu-baseline-seconds 0" "gnn-z4-bf16 --steps 10 --cpu-baseline-seconds 0" "gnn-z4 --steps 10 --cpu-baseline-seconds 0"
