# A/B of one library under two environment settings, interleaved, two rounds.
# usage: TAG=x bash tools/gpu_ab_env.sh "VAR=a" "VAR=b" <bench args>
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/abenv_${TAG:-x}; mkdir -p $O
EA=$1; EB=$2; shift 2
run() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  env $ev timeout -k 10 200 python3 bench.py --cpu-baseline-seconds 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag rc=$?"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$ev', round(d['value']), 'cw/s', round(d['ms_per_step'],3), 'ms/step')"
}
for r in 1 2; do run a_$r "$EA" "$@"; run b_$r "$EB" "$@"; done
