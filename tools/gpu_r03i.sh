# Round 3: fp32 GNN MLP on bf16x6 splits (gnn_mlp2s_kernel) -- parity, A/B vs the fp32-MFMA kernel
# (LDPC_GNN_SPLIT=0) and a 2-wave variant, kernel breakdown of cfg4 and of the training step.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_depth_gpu.py tests/test_gnn_gpu.py tests/test_train_gpu.py tests/test_custom_gnn_gpu.py tests/test_gnn_adjacency_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
V=ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib
run() {  # name, env..., -- args
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'frac', r['frac'], 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'))"
}
BA="--workload gnn-z32 --steps 3 --warmup 1"
run split LDPC_GNN_SPLIT=1
run native LDPC_GNN_SPLIT=0
run split_w2 LDPC_GNN_SPLIT=1 LDPC_AMD_LIB=$PWD/$V/variants/s2w.so
BA="--workload gnn-train-z32 --steps 10 --warmup 2"
run train_split LDPC_GNN_SPLIT=1
run train_native LDPC_GNN_SPLIT=0
BA="--workload hybrid-gnn-z32 --steps 3 --warmup 1"
run hyb_split LDPC_GNN_SPLIT=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_gnn -o run -- python3 $R/bench.py --workload gnn-z32 --steps 2 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof_gnn.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_train -o run -- python3 $R/bench.py --workload gnn-train-z32 --steps 5 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof_train.log 2>&1 || exit 1
echo prof ok
