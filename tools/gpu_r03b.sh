# debug: BP pair vs fixed; packed-add denormal semantics; then the min-sum A/B + stamped profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 60 ./tools/ubench/pk_denorm > $O/pk_denorm.log 2>&1; echo "pk rc=$?"; cat $O/pk_denorm.log
timeout -k 10 300 python tools/debug_pair_bp.py > $O/debug_pair_bp.log 2>&1; rc=$?; cat $O/debug_pair_bp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_flood_gpu.py tests/test_custom_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_flood.log 2>&1; rc=$?
tail -12 $O/pytest_flood.log
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
