set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_profile.sh gnn-z32-bf16-i10 r04a --batch 8192 || exit 1
