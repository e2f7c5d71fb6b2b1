# Sweep the GNN chunk size (frames per native launch): working-set / cache-residency effects.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/chunk_sweep2; mkdir -p $OUT
for W in gnn-z32-bf16 gnn-z32; do
for C in 512 1024 1536 2048 3072 4096 8192; do
  export LDPC_GNN_CHUNK=$C
  timeout -k 10 200 python3 $R/bench.py --workload $W --steps 3 --warmup 1 --batch 8192 --cpu-baseline-seconds 0 > $OUT/${W}_${C}.json 2> $OUT/${W}_${C}.err || { rc=$?; echo "rc=$rc at $W $C"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$OUT/${W}_${C}.json')); print('$W', $C, round(d['value']), 'cw/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done; done
