# Round 3: cfg5 early-termination overhead -- list append instead of a compaction pass, the syndrome's
# sums from LDS and a variable-major msg_out; tests, one vs two streams, one-stream breakdown
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gnn_et_gpu.py tests/test_gnn_depth_gpu.py tests/test_gnn_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'L', d.get('avg_layers'), 'ber', d.get('ber'), 'fer', d.get('fer'))"
}
BA="--workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1"
run cw_s2 LDPC_GNN_STREAMS=2
run cw_s1 LDPC_GNN_STREAMS=1
BA="--workload gnn-z32-bf16 --steps 3 --warmup 1"
run zero_s2 LDPC_GNN_STREAMS=2
BA="--workload gnn-z32-bf16-i10 --steps 3 --warmup 1"
run i10_s2 LDPC_GNN_STREAMS=2
run i10_s1 LDPC_GNN_STREAMS=1
cd /tmp && export TMPDIR=/tmp
LDPC_GNN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_s1 -o run -- python3 $R/bench.py --workload gnn-z32-bf16 --data codewords --steps 2 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof_s1.log 2>&1 || exit 1
echo prof ok
