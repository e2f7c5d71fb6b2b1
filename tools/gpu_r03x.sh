# Round 3: training weight-gradient outer products specialised for H = 64 -- gradient tests, A/B, breakdown
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --cpu-baseline-seconds 0 $BA > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'frac', round(r['frac'],3), 'kern_ms', round(r['kernel_ms'],3))"
}
BA="--workload gnn-train-z32 --steps 10 --warmup 2"
for rep in 1 2; do
  run h64_$rep LDPC_GNN_OUTER_H64=1
  run gen_$rep LDPC_GNN_OUTER_H64=0
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_train -o run -- python3 $R/bench.py --workload gnn-train-z32 --steps 5 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof_train.log 2>&1 || exit 1
echo prof ok
