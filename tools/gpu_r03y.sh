# Round 3: software-pipelined H=64 weight-gradient kernels (both / J=128 only / none) -- tests, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'frac', round(r['frac'],3), 'kern_ms', round(r['kernel_ms'],3))"
}
BA="--workload gnn-train-z32 --steps 10 --warmup 2"
for rep in 1 2; do
  run both_$rep LDPC_GNN_STREAMS=2
  run j128_$rep LDPC_AMD_LIB=$PWD/$V/variants/pipe4.so
  run none_$rep LDPC_AMD_LIB=$PWD/$V/variants/pipe0.so
done
