set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/lay_ab
for V in 0 1; do
  LDPC_GATHER_SUM_LDS=$V timeout -k 10 200 python3 bench.py --workload lay-z32 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/lay_ab/v$V.json 2> gpurun_out/lay_ab/v$V.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/lay_ab/v$V.json')); print('sum_lds=$V', round(d['value']))"
done
LDPC_GATHER_SUM_LDS=1 timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -m gpu -x -q -p no:cacheprovider 2>&1 | tail -1
