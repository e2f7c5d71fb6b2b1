# Round 3: the 6-wave kernel and the rebalanced 4-wave schedule vs the previous schedule (A/B), flood
# tests; bf16 GNN projected rows vs group means (A/B) and the bf16 tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_flood_gpu.py tests/test_gnn_et_gpu.py tests/test_gnn_depth_gpu.py tests/test_gnn_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_flood.log 2>&1; rc=$?
tail -4 $O/pytest_flood.log; [ $rc -eq 0 ] || exit $rc
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
one() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --cpu-baseline-seconds 0 --steps 30 $BA > $O/$n.json || exit $?
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,4), 'Mcw/s kern', round(d['roofline'].get('kernel_ms', 0),4), 'ber', d['ber'], d.get('avg_layers'))"
}
for rep in 1 2; do
  one fixed_$rep LDPC_FLOOD_W6=0
  one oldsched_$rep LDPC_AMD_LIB=$PWD/$V/variants/oldsched.so
  one w6_$rep LDPC_FLOOD_W6=1
done
BA="--workload bp-z32" one bp_fixed LDPC_FLOOD_W6=0
BA="--workload bp-z32" one bp_w6 LDPC_FLOOD_W6=1
for rep in 1 2; do
  BA="--workload gnn-z32-bf16-i10 --steps 5" one bf16_gm_$rep LDPC_GNN_BF16_PROJ=0
  BA="--workload gnn-z32-bf16-i10 --steps 5" one bf16_proj_$rep LDPC_GNN_BF16_PROJ=1
  BA="--workload gnn-z32-bf16-i10 --steps 5" one bf16_proj768_$rep LDPC_GNN_BF16_PROJ=1 LDPC_GNN_BF16_MLP=0
done
BA="--workload gnn-z32-bf16 --steps 5" one cfg5_gm LDPC_GNN_BF16_PROJ=0
BA="--workload gnn-z32-bf16 --steps 5" one cfg5_proj LDPC_GNN_BF16_PROJ=1
LDPC_FLOOD_W6=1 bash tools/gpu_profile.sh minsum-z32 r03d_w6 || exit 1
