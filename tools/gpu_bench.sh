# usage: bash tools/gpu_bench.sh <tag> <workload> [bench args...]   (bench + kernel-trace stats)
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; W=$2; shift 2
OUT=$R/gpurun_out/bench_${TAG}_${W}; mkdir -p $OUT
timeout -k 10 400 python3 $R/bench.py --workload $W "$@" > $OUT/bench.json 2> $OUT/bench.err || { rc=$?; echo "bench rc=$rc"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload $W --steps 5 --warmup 1 --cpu-baseline-seconds 0 "$@" > $OUT/trace.log 2>&1; echo "trace rc=$?"
cat $OUT/bench.json
