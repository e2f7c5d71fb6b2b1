set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/layers; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -25 $OUT/pytest.log; exit $rc
