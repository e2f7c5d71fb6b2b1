# Round 3, first GPU pass: flood tests (incl. the frame-pair kernel), A/B of the min-sum kernels
# on cfg3, then the stamped rocprof + PMC passes of the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_flood_gpu.py tests/test_custom_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_flood.log 2>&1; rc=$?
tail -5 $O/pytest_flood.log; [ $rc -eq 0 ] || exit $rc
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
one() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --cpu-baseline-seconds 0 --steps 30 $BA > $O/$n.json || exit $?
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,2), 'Mcw/s kern', round(d['roofline']['kernel_ms'],4), 'ber', d['ber'])"
}
for rep in 1 2; do
  one pair_$rep LDPC_FLOOD_PAIR=1
  one fixed_min3_$rep LDPC_FLOOD_PAIR=0
  one fixed_old_$rep LDPC_FLOOD_PAIR=0 LDPC_AMD_LIB=$PWD/$V/variants/min3off.so
done
BA="--workload bp-z32" one bp_pair LDPC_FLOOD_PAIR=1
BA="--workload bp-z32" one bp_fixed LDPC_FLOOD_PAIR=0
bash tools/gpu_profile.sh minsum-z32 r03a
