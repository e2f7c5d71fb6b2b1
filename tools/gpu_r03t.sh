# Round 3: split MLP with the next tile's feature rows prefetched (2 waves/SIMD) vs default (3 waves)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03t; mkdir -p $O
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
LDPC_AMD_LIB=$PWD/$V/variants/s2pf.so timeout -k 10 600 python -u -m pytest tests/test_gnn_depth_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider -k "cfg4" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3))"
}
BA="--workload gnn-z32 --steps 3 --warmup 1"
for rep in 1 2; do
  run def_$rep LDPC_GNN_STREAMS=2
  run pf_$rep LDPC_AMD_LIB=$PWD/$V/variants/s2pf.so
done
