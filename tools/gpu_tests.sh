# GPU test pass: smoke, then every -m gpu test (verbose, per-test timeout), logs under gpurun_out/.
# usage (on the box via gpurun): bash tools/gpu_tests.sh [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rP --timeout 240 --timeout-method thread -p no:cacheprovider "${K[@]}" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
