# several bench lines in one session: bash tools/gpu_multi.sh <tag> "<workload> [args]" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; shift
OUT=$R/gpurun_out/multi_${TAG}; mkdir -p $OUT
i=0
for spec in "$@"; do
  i=$((i+1))
  timeout -k 10 500 python3 $R/bench.py --workload $spec > $OUT/run$i.json 2> $OUT/run$i.err || { rc=$?; echo "run $i ($spec) rc=$rc"; tail -5 $OUT/run$i.err; exit $rc; }
  echo "$spec: $(python3 -c "import json;d=json.load(open('$OUT/run$i.json'));print(round(d['value'],1),'cw/s', round(d['ms_per_step'],3),'ms', 'frac', round(d['roofline']['frac'],3))")"
done
