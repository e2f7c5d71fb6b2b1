# Generic speed-knob A/B: KNOB=<env var> VARIANTS="a b ..." WORKLOAD=<bench workload> [BATCH, STEPS]
# runs the workload once per value (results are identical across the speed-only knobs).
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/knob_ab; mkdir -p $OUT
cd $R
for V in ${VARIANTS:?}; do
  env "${KNOB:?}=$V" timeout -k 10 200 python3 bench.py --workload ${WORKLOAD:?} --steps ${STEPS:-3} --warmup 1 ${BATCH:+--batch $BATCH} --cpu-baseline-seconds 0 > $OUT/v$V.json 2> $OUT/v$V.err || { echo "bench rc=$? v$V"; tail -5 $OUT/v$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/v$V.json')); print('$KNOB=$V', round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms frac', round(d['roofline']['frac'],3), 'ber', d.get('ber'))"
done
