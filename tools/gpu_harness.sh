set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/harness; mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_harness_gpu.py tests/test_layers_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -30 $OUT/pytest.log; exit $rc
