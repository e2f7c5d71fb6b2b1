set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab
O=gpurun_out/ab
V=$GRAFT_REPO_ROOT/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/variants
run() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python3 bench.py --cpu-baseline-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],4), 'ms', 'ber', d.get('ber'))"
}
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -q -rP --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sub.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  run fp32_main_$r X=1 --workload gnn-z32 --steps 3 --warmup 1 || exit 1
  run fp32_noslp_$r LDPC_AMD_LIB=$V/noslp_gnn.so --workload gnn-z32 --steps 3 --warmup 1 || exit 1
  run fp32_restr512_$r LDPC_AMD_LIB=$V/restr512.so --workload gnn-z32 --steps 3 --warmup 1 || exit 1
  run fp32_restr512n_$r LDPC_AMD_LIB=$V/restr512_noslp.so --workload gnn-z32 --steps 3 --warmup 1 || exit 1
  run hyb_main_$r X=1 --workload hybrid-gnn-z32 --steps 3 --warmup 1 || exit 1
  run hyb_noslp_$r LDPC_AMD_LIB=$V/noslp_gnn.so --workload hybrid-gnn-z32 --steps 3 --warmup 1 || exit 1
  run hyb_restr512n_$r LDPC_AMD_LIB=$V/restr512_noslp.so --workload hybrid-gnn-z32 --steps 3 --warmup 1 || exit 1
  run i10_main_$r X=1 --workload gnn-z32-bf16-i10 --steps 3 --warmup 1 || exit 1
  run i10_noslp_$r LDPC_AMD_LIB=$V/noslp_bf16.so --workload gnn-z32-bf16-i10 --steps 3 --warmup 1 || exit 1
  run train_main_$r X=1 --workload gnn-train-z32 --steps 5 --warmup 2 || exit 1
  run train_noslp_$r LDPC_AMD_LIB=$V/noslp_train.so --workload gnn-train-z32 --steps 5 --warmup 2 || exit 1
done
