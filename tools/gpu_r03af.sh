# Round 3: cfg5 early-termination overhead -- lists vs flags, one vs two streams; one-stream breakdown
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03af; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'L', d.get('avg_layers'))"
}
BA="--workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1"
run s2_list LDPC_GNN_STREAMS=2
run s2_flags LDPC_GNN_STREAMS=2 LDPC_GNN_ET_COMPACT=0
run s1_list LDPC_GNN_STREAMS=1
cd /tmp && export TMPDIR=/tmp
LDPC_GNN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_s1 -o run -- python3 $R/bench.py --workload gnn-z32-bf16 --data codewords --steps 1 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/trace_s1.log 2>&1 || exit 1
echo trace ok
