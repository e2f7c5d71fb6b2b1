# One GPU call: smoke + the whole -m gpu suite, then (unless a test run died: fault, abort, timeout)
# an interleaved A/B of one workload against ab/<variant>.so, then optional profiles.
# usage: TAG=x AB="<variants>" BENCH="<bench args>" PROF="<workload> ..." bash tools/gpu_check_ab.sh [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu_tests.sh "$1"; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
if [ -n "$AB" ]; then TAG=${TAG:-x} bash tools/gpu_ab.sh "$AB" "" $BENCH || exit $?; fi
for w in $PROF; do bash tools/gpu_profile.sh $w ${TAG:-x} || exit $?; done
exit $rc
