# Round-5 refresh after the f16 MLP: profiles + stamped PMC summaries of the fp32 GNN forward and the
# training step (the workloads whose kernels changed), then every bench line.
# usage: TAG=r05y bash tools/gpu_evidence_y.sh [profile|bench]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${TAG:-r05y}; O=$R/gpurun_out/evidence_$T; mkdir -p $O
summ() {  # workload kernel-substring per-call-kernel batch note
  local W=$1 K=$2 PC=$3 B=$4 N=$5 w=${1//-/_}
  python3 tools/pmc_summary.py gpurun_out/prof_${T}_${W} "$K" profiles/${T}_pmc_${w}.json - $PC > /dev/null || return 1
  python3 - profiles/${T}_pmc_${w}.json "$B" "$N" <<'PY' || return 1
import json, sys
f, b, note = sys.argv[1], float(sys.argv[2]), sys.argv[3]
d = json.load(open(f)); d["batch"] = b; d["note"] = note
json.dump(d, open(f, "w"), indent=1)
PY
  cp profiles/${T}_pmc_${w}.json $O/
  mkdir -p $O/prof_${W}
  cp gpurun_out/prof_${T}_${W}/trace/run_kernel_stats.csv $O/prof_${W}/kernel_stats.csv
  cp gpurun_out/prof_${T}_${W}/lib_sha256.txt gpurun_out/prof_${T}_${W}/code_objects_sha256.txt $O/prof_${W}/
  python3 tools/pmc_kernels.py gpurun_out/prof_${T}_${W} > $O/prof_${W}/pmc_per_kernel.txt || true
}
if [ "${1:-profile}" = profile ]; then
  bash tools/gpu_profile.sh gnn-z32 $T > $O/prof_gnn-z32.log 2>&1 || exit 1
  summ gnn-z32 "gnn_|csr_" csr_count_kernel 10922.666666666666 "per call = one fp32 GNN forward call on one workspace chunk (bench's B=32768 runs as 3 chunks of ~10923 frames); every gnn_*/csr_* kernel of the call summed, divided by the csr_count_kernel launches (one per call)" || exit 1
  bash tools/gpu_profile.sh gnn-train-z32 $T > $O/prof_gnn-train-z32.log 2>&1 || exit 1
  summ gnn-train-z32 "train_|gnn_|csr_" train_head_kernel 256 "per call = one gnn-train-z32 step (fp32 forward saving features and projections, BCE, HIP backward of 10 layers, SGD) on 256 frames; every train_*/gnn_*/csr_* kernel of the step summed, divided by the train_head_kernel launches (one per step)" || exit 1
  echo "profiles ok"
else
  bash tools/gpu_bench_all.sh || exit $?
  mkdir -p $O/bench_all && cp gpurun_out/bench_all/*.json $O/bench_all/
fi
