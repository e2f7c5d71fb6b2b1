# Copy a round-end GPU run (tools/gpu_round_end.sh) from gpurun_out/ into profiles/<TAG>_*.
# usage: bash tools/collect_profiles.sh <TAG>
set -e
T=${1:?tag}
cd "$(dirname "$0")/.."
for W in minsum-z32 gnn-z32-bf16-i10; do
  w=${W//-/_}; P=gpurun_out/prof_${T}_${W}
  mkdir -p profiles/${T}_pmc_${w}
  for i in 1 2 3 4; do cp $P/pmc$i/run_counter_collection.csv profiles/${T}_pmc_${w}/pmc$i.csv; done
  cp $P/trace/run_kernel_stats.csv profiles/${T}_rocprof_stats_${w}.csv
done
python3 tools/pmc_summary.py gpurun_out/prof_${T}_minsum-z32 flood_fixed profiles/${T}_pmc_minsum_z32.json 436207616 > /dev/null
python3 tools/pmc_summary.py gpurun_out/prof_${T}_gnn-z32-bf16-i10 "gnn_|csr_" profiles/${T}_pmc_gnn_z32_bf16_i10.json - gnn_bf16_info_kernel > /dev/null
python3 - "$T" <<'PY'
import json, sys
t = sys.argv[1]
for f, b, note in ((f"profiles/{t}_pmc_minsum_z32.json", 65536, None),
                   (f"profiles/{t}_pmc_gnn_z32_bf16_i10.json", 8192,
                    "per call = one 10-layer bf16 GNN forward (every gnn_*/csr_* kernel of the call summed, "
                    "divided by the gnn_bf16_info_kernel launches); batch 8192 frames")):
    d = json.load(open(f)); d["batch"] = b
    if note: d["note"] = note
    json.dump(d, open(f, "w"), indent=1)
PY
for f in gpurun_out/bench_all/*.json; do n=$(basename $f .json); cp $f profiles/${T}_bench_${n//-/_}.json; done
cp gpurun_out/pytest_gpu.log profiles/${T}_pytest_gpu.log
ls profiles | grep "^${T}_" | wc -l
