# A/B timing of the GNN forward's stream split and MLP occupancy knobs (env vars, same library),
# after the GNN parity tests.  usage: bash tools/gpu_ab_gnn.sh [tests=1]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abg
if [ "${1:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gnn_gpu.py tests/test_gnn_et_gpu.py tests/test_gnn_depth_gpu.py tests/test_gnn_adjacency_gpu.py \
    tests/test_train_gpu.py > gpurun_out/abg/pytest.log 2>&1 || { tail -30 gpurun_out/abg/pytest.log; exit 1; }
  tail -2 gpurun_out/abg/pytest.log
fi
run() {  # name workload env...
  n=$1; wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --workload $wl --cpu-baseline-seconds 0 --steps 3 --warmup 1 > gpurun_out/abg/$n.json || exit $?
  echo "$n $(python -c "import json; d=json.load(open('gpurun_out/abg/$n.json')); print(round(d['value'],0), 'cw/s ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],3))")"
}
V=$PWD/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/variants
for rep in ${REPS:-1 2}; do
  for c in ${CASES:-fp32_proj:gnn-z32:LDPC_GNN_STREAMS=2 fp32_noproj:gnn-z32:LDPC_GNN_PROJ=0}; do
    IFS=: read n wl envs <<< "$c"; run $n $wl ${envs//,/ }
  done
  for v in $(ls $V 2>/dev/null | sed 's/\.so$//'); do run fp32_$v gnn-z32 LDPC_AMD_LIB=$V/$v.so; done
done
if [ -n "$PROF" ]; then  # one single-stream kernel-trace pass of the fp32 forward
  cd /tmp && export TMPDIR=/tmp
  LDPC_GNN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/abg/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload ${PROF} --steps 3 --warmup 1 --cpu-baseline-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/abg/trace.log 2>&1 || exit $?
fi
