# Round-6 evidence: profiles + stamped PMC summaries of the workloads whose kernels changed this round
# (the headline min-sum kernel is re-profiled on the same box as its bench line), then every bench line.
# usage: TAG=r06 bash tools/gpu_evidence_r06.sh [profile|bench]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${TAG:-r06}; O=$R/gpurun_out/evidence_$T; mkdir -p $O
summ() {  # workload kernel-substring per-call-kernel|- batch expected-read|- note
  local W=$1 K=$2 PC=$3 B=$4 X=$5 N=$6 w=${1//-/_}
  if [ "$PC" = "-" ]; then
    python3 tools/pmc_summary.py gpurun_out/prof_${T}_${W} "$K" profiles/${T}_pmc_${w}.json $X > /dev/null || return 1
  else
    python3 tools/pmc_summary.py gpurun_out/prof_${T}_${W} "$K" profiles/${T}_pmc_${w}.json $X $PC > /dev/null || return 1
  fi
  python3 - profiles/${T}_pmc_${w}.json "$B" "$N" <<'PY' || return 1
import json, sys
f, b, note = sys.argv[1], float(sys.argv[2]), sys.argv[3]
d = json.load(open(f)); d["batch"] = b
if note: d["note"] = note
json.dump(d, open(f, "w"), indent=1)
PY
  cp profiles/${T}_pmc_${w}.json $O/
  mkdir -p $O/prof_${W}
  cp gpurun_out/prof_${T}_${W}/trace/run_kernel_stats.csv $O/prof_${W}/kernel_stats.csv
  cp gpurun_out/prof_${T}_${W}/lib_sha256.txt gpurun_out/prof_${T}_${W}/code_objects_sha256.txt $O/prof_${W}/
  cp gpurun_out/prof_${T}_${W}/trace_bench.log $O/prof_${W}/trace_bench.json 2>/dev/null || true
  python3 tools/pmc_kernels.py gpurun_out/prof_${T}_${W} > $O/prof_${W}/pmc_per_kernel.txt || true
}
if [ "${1:-profile}" = profile ]; then
  # WL: the workloads to profile (default: all six)
  for w in ${WL:-minsum-z32 gnn-z4 gnn-z32 gnn-z32-h128 gnn-z32-bf16-i10 gnn-z32-bf16}; do
    bash tools/gpu_profile.sh $w $T > $O/prof_$w.log 2>&1 || exit 1
    case $w in
      minsum-z32) summ minsum-z32 flood_fixed - 65536 436207616 "" || exit 1 ;;
      gnn-z4) summ gnn-z4 "gnn_|csr_" csr_count_kernel 4096 - "per call = one 5-layer fp32 GNN forward on B=4096 Z=4 frames (cfg2); every gnn_*/csr_* kernel of the call summed, divided by the csr_count_kernel launches (one per call)" || exit 1 ;;
      gnn-z32) summ gnn-z32 "gnn_|csr_" csr_count_kernel 10922.666666666666 - "per call = one fp32 GNN forward call on one workspace chunk (bench's B=32768 runs as 3 chunks of ~10923 frames); every gnn_*/csr_* kernel of the call summed, divided by the csr_count_kernel launches (one per call)" || exit 1 ;;
      gnn-z32-h128) summ gnn-z32-h128 "gnn_|csr_" csr_count_kernel 2730.6666666666665 - "per call = one H=128 fp32 GNN forward call on one workspace chunk (B=8192 runs as 3 chunks); every gnn_*/csr_* kernel of the call summed, divided by the csr_count_kernel launches (one per call)" || exit 1 ;;
      gnn-z32-bf16-i10) summ gnn-z32-bf16-i10 "gnn_|csr_" gnn_bf16_info_kernel 16384 - "per call = one 10-layer bf16 GNN forward on one 16384-frame chunk (B=32768 runs as 2 chunks); every gnn_*/csr_* kernel of the call summed, divided by the gnn_bf16_info_kernel launches (one per call)" || exit 1 ;;
      gnn-z32-bf16) summ gnn-z32-bf16 "gnn_|csr_" gnn_bf16_info_kernel 16384 - "per call = one 15-layer bf16 GNN forward with per-frame early termination on one 16384-frame chunk (B=32768 runs as 2 chunks), random codewords at 2 dB; every gnn_*/csr_* kernel of the call summed, divided by the gnn_bf16_info_kernel launches (one per call)" || exit 1 ;;
    esac
  done
  echo "profiles ok"
else
  bash tools/gpu_bench_all.sh || exit $?
  mkdir -p $O/bench_all && cp gpurun_out/bench_all/*.json $O/bench_all/
  # the headline kernel under rocprof on the same box, right after its plain bench line
  mkdir -p $O/headline && cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/headline/trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 > $O/headline/bench_under_rocprof.json 2> $O/headline/rocprof.err || exit $?
  cd $R && timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 > $O/headline/bench_after.json 2>/dev/null || exit $?
  echo "headline ok"
fi
