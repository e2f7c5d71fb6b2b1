# Round-end evidence in one GPU call: rocprof kernel statistics + PMC passes of every workload whose
# bench line carries measured HBM traffic, their stamped summaries (written into the box's copy of
# profiles/ so that the bench lines that follow find them, and into gpurun_out/evidence/), then
# every bench line.  usage: TAG=r05x bash tools/gpu_evidence.sh [profile|bench|all]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${TAG:-r05x}; O=$R/gpurun_out/evidence; mkdir -p $O
WHAT=${1:-all}
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
# PART=1 / PART=2: the first three / the last three workloads (one GPU call each)
P1=true; P2=true
[ "${PART:-}" = 1 ] && P2=false
[ "${PART:-}" = 2 ] && P1=false
if { [ "$WHAT" = all ] || [ "$WHAT" = profile ]; } && $P1; then
  bash tools/gpu_profile.sh gnn-z32 $T > $O/prof_gnn-z32.log 2>&1 || exit 1
  summ gnn-z32 "gnn_|csr_" csr_count_kernel 10922.666666666666 "per call = one fp32 GNN forward call on one workspace chunk (bench's B=32768 runs as 3 chunks of ~10923 frames); every gnn_*/csr_* kernel of the call summed, divided by the csr_count_kernel launches (one per call)" || exit 1
  bash tools/gpu_profile.sh gnn-z32-bf16 $T > $O/prof_gnn-z32-bf16.log 2>&1 || exit 1
  summ gnn-z32-bf16 "gnn_|csr_" gnn_bf16_info_kernel 16384 "per call = one 15-layer bf16 GNN forward with per-frame early termination on one 16384-frame chunk (B=32768 runs as 2 chunks), random codewords at 2 dB; every gnn_*/csr_* kernel of the call summed, divided by the gnn_bf16_info_kernel launches (one per call)" || exit 1
  bash tools/gpu_profile.sh gnn-z32-bf16-i10 $T > $O/prof_gnn-z32-bf16-i10.log 2>&1 || exit 1
  summ gnn-z32-bf16-i10 "gnn_|csr_" gnn_bf16_info_kernel 16384 "per call = one 10-layer bf16 GNN forward on one 16384-frame chunk (B=32768 runs as 2 chunks); every gnn_*/csr_* kernel of the call summed, divided by the gnn_bf16_info_kernel launches (one per call)" || exit 1
  echo "profiles part 1 ok"
fi
if { [ "$WHAT" = all ] || [ "$WHAT" = profile ]; } && $P2; then
  bash tools/gpu_profile.sh gnn-z32-h128 $T > $O/prof_gnn-z32-h128.log 2>&1 || exit 1
  summ gnn-z32-h128 "gnn_|csr_" csr_count_kernel 2730.6666666666665 "per call = one H=128 fp32 GNN forward call on one workspace chunk (B=8192 runs as 3 chunks); every gnn_*/csr_* kernel of the call summed, divided by the csr_count_kernel launches (one per call)" || exit 1
  bash tools/gpu_profile.sh gnn-train-z32 $T > $O/prof_gnn-train-z32.log 2>&1 || exit 1
  summ gnn-train-z32 "train_|gnn_|csr_" train_head_kernel 256 "per call = one gnn-train-z32 step (fp32 forward saving features and projections, BCE, HIP backward of 10 layers, SGD) on 256 frames; every train_*/gnn_*/csr_* kernel of the step summed, divided by the train_head_kernel launches (one per step)" || exit 1
  bash tools/gpu_profile.sh lay-z32 $T > $O/prof_lay-z32.log 2>&1 || exit 1
  summ lay-z32 "check_group|var_group|residual|output_layer" output_layer_kernel 4096 "per call = one lay-z32 step (10 iterations of CheckLayer -> VariableLayer -> ResidualLayer, then OutputLayer) on 4096 frames; every check_group/var_group/residual/output_layer kernel of the step summed, divided by the output_layer_kernel launches (one per step)" || exit 1
  echo "profiles ok"
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  bash tools/gpu_bench_all.sh || exit $?
  mkdir -p $O/bench_all && cp gpurun_out/bench_all/*.json $O/bench_all/
fi
