# Train the Z=32 MessageGNN checkpoints (15 layers for cfg5, 10 layers for cfg4) with the HIP
# trainer, then bench the GNN lines with them.  Checkpoints land in gpurun_out/ckpt/ (copy them to
# checkpoints/ to keep).  usage: bash tools/gpu_train.sh [minutes15] [minutes10]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/train; C=gpurun_out/ckpt; mkdir -p $O $C
M15=${1:-7}; M10=${2:-5}
timeout -k 10 60 rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
timeout -k 10 $((M15 * 60 + 240)) python -u tools/train_gnn_checkpoint.py --layers 15 --minutes $M15 \
  --out $C/gnn_bg2_z32_i15_h64.pt > $O/train_i15.log 2>&1 || { tail -20 $O/train_i15.log; exit 1; }
tail -3 $O/train_i15.log
timeout -k 10 $((M10 * 60 + 240)) python -u tools/train_gnn_checkpoint.py --layers 10 --minutes $M10 \
  --out $C/gnn_bg2_z32_i10_h64.pt > $O/train_i10.log 2>&1 || { tail -20 $O/train_i10.log; exit 1; }
tail -3 $O/train_i10.log
B="timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --steps 5 --warmup 1"
$B --workload gnn-z32-bf16 --checkpoint $C/gnn_bg2_z32_i15_h64.pt > $O/gnn_z32_bf16.json || exit 1
$B --workload gnn-z32 --checkpoint $C/gnn_bg2_z32_i10_h64.pt > $O/gnn_z32.json || exit 1
$B --workload gnn-z32-bf16-i10 --checkpoint $C/gnn_bg2_z32_i10_h64.pt > $O/gnn_z32_bf16_i10.json || exit 1
for s in 0 1 3 4; do
  $B --workload gnn-z32-bf16 --snr $s --checkpoint $C/gnn_bg2_z32_i15_h64.pt > $O/gnn_z32_bf16_snr$s.json || exit 1
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), 'cw/s', 'ber', d['ber'], 'fer', d['fer'], 'avg_layers', d['avg_layers'])"; done
