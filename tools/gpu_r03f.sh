# Round 3: training backward from projected group rows (parity + A/B + kernel times)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=$PWD/gpurun_out/r03f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for pj in 1 0; do
    LDPC_GNN_TRAIN_PROJ=$pj timeout -k 10 120 python bench.py --workload gnn-train-z32 --steps 20 --cpu-baseline-seconds 0 > $O/train_pj${pj}_$rep.json || exit 1
    python -c "import json; d=json.load(open('$O/train_pj${pj}_$rep.json')); print('pj$pj', round(d['value']), round(d['ms_per_step'],2), d['roofline']['frac'])"
  done
done
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload gnn-train-z32 --steps 5 --warmup 1 --cpu-baseline-seconds 0 > $O/prof.json 2> $O/prof.err || exit 1
echo prof ok
