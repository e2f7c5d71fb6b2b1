# Round 3: full GPU suite + smoke + training line after the side-stream backward default
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03ak; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload gnn-train-z32 > $O/gnn_train_z32.json 2> $O/gnn_train_z32.err || exit $?
python3 -c "import json; d=json.load(open('$O/gnn_train_z32.json')); print(round(d['value']), d['ms_per_step'], d['roofline']['frac'])"
