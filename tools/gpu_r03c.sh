# Round 3: full -m gpu suite, min-sum kernel A/B (fixed default, MIN3 off, compare-free select,
# frame-pair kernel), stamped rocprof + PMC of the default build and of the pair kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -8 $O/pytest_gpu.log
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
one() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --cpu-baseline-seconds 0 --steps 30 $BA > $O/$n.json || exit $?
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,2), 'Mcw/s kern', round(d['roofline']['kernel_ms'],4), 'ber', d['ber'])"
}
for rep in 1 2; do
  one fixed_$rep LDPC_FLOOD_PAIR=0
  one min3off_$rep LDPC_AMD_LIB=$PWD/$V/variants/min3off.so
  one selfree_$rep LDPC_AMD_LIB=$PWD/$V/variants/selfree.so
  one pair_$rep LDPC_FLOOD_PAIR=1
done
BA="--workload bp-z32" one bp_fixed LDPC_FLOOD_PAIR=0
BA="--workload bp-z32" one bp_pair LDPC_FLOOD_PAIR=1
bash tools/gpu_profile.sh minsum-z32 r03c || exit 1
LDPC_FLOOD_PAIR=1 bash tools/gpu_profile.sh minsum-z32 r03c_pair || exit 1
exit $rc
