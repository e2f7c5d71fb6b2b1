# Round 3: streaming decoder throughput vs batch (does an Infinity-Cache-sized batch run faster?)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03o; mkdir -p $O
for b in 65536 16384 8192 4096 2048; do
  timeout -k 10 120 python3 bench.py --workload minsum-z32-stream --batch $b --steps 20 --warmup 3 --cpu-baseline-seconds 0 > $O/s_$b.json 2> $O/s_$b.err || exit 1
  python3 -c "import json; d=json.load(open('$O/s_$b.json')); r=d['roofline']; print('B=$b', round(d['value']), 'frac', r['frac'], 'kern_ms', round(r['kernel_ms'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof8k -o run -- python3 $R/bench.py --workload minsum-z32-stream --batch 8192 --steps 5 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof8k.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof64k -o run -- python3 $R/bench.py --workload minsum-z32-stream --steps 5 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof64k.log 2>&1 || exit 1
echo prof ok
