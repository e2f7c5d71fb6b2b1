# rocprof kernel stats + PMC passes for the flood workloads (minsum-z32 = cfg3, bp-z32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r02}
bash tools/gpu_profile.sh minsum-z32 $T && bash tools/gpu_profile.sh bp-z32 $T
