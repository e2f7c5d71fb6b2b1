# A/B timing of library variants on the cfg3 bench (min-sum Z=32, B=65536, 10 it) and BP Z=32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
for rep in 1 2; do
for n in base $(ls $V/variants | sed 's/\.so$//'); do
  lib=$V/libldpc_amd.so; [ $n != base ] && lib=$V/variants/$n.so
  LDPC_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --cpu-baseline-seconds 0 --steps 30 > gpurun_out/ab/$n.json || exit $?
  echo "$rep $n $(python -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print(round(d['value']/1e6,2), 'Mcw/s kern', round(d['roofline']['kernel_ms'],4))")"
done; done
