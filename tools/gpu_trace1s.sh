# One-stream kernel trace (rocprofv3 --kernel-trace --stats) of bench workloads: per-kernel times
# without the two-stream co-scheduling.  usage: TAG=x bash tools/gpu_trace1s.sh <workload> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; W=$1; shift
O=$R/gpurun_out/tr1s_${TAG:-x}_$W
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LDPC_GNN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --workload $W --cpu-baseline-seconds 0 "$@" > $O/bench.log 2>&1 || { echo "trace $W rc=$?"; exit 1; }
python3 - $O/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if float(r["Percentage"]) >= 0.5:
        print(f'{r["Name"][:70]:70s} {r["Calls"]:>6} {float(r["AverageNs"])/1e3:10.1f} us {float(r["Percentage"]):6.2f} %')
PY
