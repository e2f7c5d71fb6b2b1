# gpu tests (all) then an A/B bench: bash tools/gpu_test_ab.sh <tag> <workload> "<ENV>" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; W=$2; shift 2
mkdir -p $R/gpurun_out
timeout -k 10 900 python -m pytest $R/tests -m gpu -q -p no:cacheprovider -x > $R/gpurun_out/pytest_${TAG}.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $R/gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash $R/tools/gpu_ab.sh $TAG $W "$@"
