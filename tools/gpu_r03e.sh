# Round 3: bf16 projected rows (parity + kernel times vs group means), training-step kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=$PWD/gpurun_out/r03e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gnn_depth_gpu.py -k "projected or cfg5" -q -s --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "proj=|passed|failed" $O/pytest.log; [ $rc -eq 0 ] || exit $rc
R=$PWD; cd /tmp && export TMPDIR=/tmp
prof() {  # tag, env..., -- bench args
  t=$1; shift; envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t -o run -- python3 $R/bench.py --cpu-baseline-seconds 0 --warmup 1 "$@" > $O/$t.json 2> $O/$t.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $O/$t.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); print('$t', round(d['value']), d['ms_per_step'], d['ber'])"
}
prof bf16p LDPC_GNN_BF16_PROJ=1 -- --workload gnn-z32-bf16-i10 --steps 3
prof bf16g LDPC_GNN_BF16_PROJ=0 -- --workload gnn-z32-bf16-i10 --steps 3
prof train LDPC_X=1 -- --workload gnn-train-z32 --steps 5
prof fp32 LDPC_X=1 -- --workload gnn-z32 --steps 3
