# A/B bench of env settings in one box session: bash tools/gpu_ab.sh <tag> <workload> "<ENV=..>" "<ENV=..>" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; W=$2; shift 2
OUT=$R/gpurun_out/ab_${TAG}; mkdir -p $OUT
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python3 $R/bench.py --workload $W --cpu-baseline-seconds 0 $BENCH_ARGS > $OUT/run$i.json 2> $OUT/run$i.err || { rc=$?; echo "run $i ($envs) rc=$rc"; exit $rc; }
  echo "$envs: $(python3 -c "import json;d=json.load(open('$OUT/run$i.json'));print(round(d['value']/1e6,3),'Mcw/s', round(d['ms_per_step'],3),'ms')")"
done
