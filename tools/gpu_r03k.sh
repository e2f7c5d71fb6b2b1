# Round 3: projection kernel workgroup size (12 / 8 / 6 waves per CU) on cfg4 (fp32, split MLP)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03k; mkdir -p $O
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'frac', r['frac'], 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'))"
}
BA="--workload gnn-z32 --steps 3 --warmup 1"
for rep in 1 2; do
  run p768_$rep LDPC_GNN_SPLIT=1
  run p512_$rep LDPC_AMD_LIB=$PWD/$V/variants/p512.so
  run p384_$rep LDPC_AMD_LIB=$PWD/$V/variants/p384.so
done
