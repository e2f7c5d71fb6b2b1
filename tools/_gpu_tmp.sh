set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_gnn_gpu.py tests/test_gnn_depth_gpu.py tests/test_custom_gnn_gpu.py tests/test_checkpoints_gpu.py -q -rP --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sub.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/ab
V=$GRAFT_REPO_ROOT/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/variants
run() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python3 bench.py --cpu-baseline-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],4), 'ms', 'ber', d.get('ber'))"
}
for r in 1 2; do
  run train_base_$r LDPC_AMD_LIB=$V/gnn_r04base.so --workload gnn-train-z32 --steps 5 --warmup 2 || exit 1
  run train_new_$r X=1 --workload gnn-train-z32 --steps 5 --warmup 2 || exit 1
  run fp32_new_$r X=1 --workload gnn-z32 --steps 3 --warmup 1 || exit 1
done
mkdir -p gpurun_out/prof_train
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train/new -o run -- python3 bench.py --workload gnn-train-z32 --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/prof_train/new.log 2>&1
