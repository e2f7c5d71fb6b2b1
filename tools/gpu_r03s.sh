# Round 3: bf16 MLP D1-table LDS stride 68 (default) vs 64 -- tests, A/B, PMC of the MLP kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_et_gpu.py tests/test_gnn_depth_gpu.py tests/test_gnn_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'L', d.get('avg_layers'))"
}
for rep in 1 2; do
  BA="--workload gnn-z32-bf16-i10 --steps 3 --warmup 1"
  run i10_d68_$rep LDPC_GNN_STREAMS=2
  run i10_d64_$rep LDPC_AMD_LIB=$PWD/$V/variants/d1s64.so
done
BA="--workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1"
run cfg5_d68 LDPC_GNN_STREAMS=2
run cfg5_d64 LDPC_AMD_LIB=$PWD/$V/variants/d1s64.so
BA="--workload gnn-z32 --steps 3 --warmup 1"
run gnn_z32_emb68 LDPC_GNN_STREAMS=2
cd /tmp && export TMPDIR=/tmp
export LDPC_GNN_STREAMS=1
B="python3 $R/bench.py --workload gnn-z32-bf16-i10 --batch 8192 --steps 1 --warmup 1 --cpu-baseline-seconds 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc2 -o run -- $B > $R/$O/pmc2.log 2>&1 || exit 1
echo pmc ok
