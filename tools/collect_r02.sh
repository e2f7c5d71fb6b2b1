# Copy a round-2 profile run (tools/gpu_profile.sh <workload> <TAG>) into profiles/<TAG>_*.
# usage: bash tools/collect_r02.sh <TAG> <workload> [batch] [kernel-substring] [expected-read-bytes|-]
set -e
T=${1:?tag}; W=${2:?workload}; B=${3:-65536}; K=${4:-flood}; X=${5:--}
cd "$(dirname "$0")/.."
w=${W//-/_}; P=gpurun_out/prof_${T}_${W}
mkdir -p profiles/${T}_pmc_${w}
for d in $P/pmc*/; do n=$(basename $d); cp $d/run_counter_collection.csv profiles/${T}_pmc_${w}/$n.csv; done
cp $P/trace/run_kernel_stats.csv profiles/${T}_rocprof_stats_${w}.csv
python3 tools/pmc_summary.py $P "$K" profiles/${T}_pmc_${w}.json $X > /dev/null
python3 - "$T" "$w" "$B" <<'PY'
import json, sys
t, w, b = sys.argv[1], sys.argv[2], int(sys.argv[3])
f = f"profiles/{t}_pmc_{w}.json"
d = json.load(open(f)); d["batch"] = b; json.dump(d, open(f, "w"), indent=1)
print(f, json.dumps(d.get("derived", {})))
PY
