# A/B on one box: the default library against variant libraries (ab/<name>.so or $VARDIR/<name>.so,
# interleaved, two rounds) on one bench workload, plus the phase timelines of flood timeline builds.
# Lines land in gpurun_out/ab_<TAG>/.
# usage: TAG=x bash tools/gpu_ab.sh "<variant names>" "<timeline names>" [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/ab_${TAG:-flood}; mkdir -p $O
V=${VARDIR:-$R/ab}
VARS=$1; TLS=$2; shift 2
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  LDPC_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --cpu-baseline-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],4), 'ms', 'layers', d.get('avg_layers'), 'ber', d.get('ber'))"
}
for r in 1 2; do
  run base_$r $R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so "$@"
  for v in $VARS; do run ${v}_$r $V/$v.so "$@"; done
done
for t in $TLS; do
  LDPC_TIMELINE_OUT=$O/$t.bin run $t $V/$t.so --steps 1 --warmup 1 "$@"
  python3 tools/flood_timeline.py $O/$t.bin $O/$t.json > /dev/null && echo "timeline $t ok"
done
