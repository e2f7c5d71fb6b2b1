# Train the Z=32 MessageGNN checkpoints (15 layers for cfg5, 10 layers for cfg4) with the HIP
# trainer, then bench the GNN lines with them (all-zero and random-codeword frames).  Checkpoints
# land in gpurun_out/ckpt/ (copy them to checkpoints/ to keep).
# usage: bash tools/gpu_train.sh [minutes15] [minutes10] [init: 1 = continue from checkpoints/]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/train; C=gpurun_out/ckpt; mkdir -p $O $C
M15=${1:-7}; M10=${2:-5}; INIT=${3:-0}
I15=""; I10=""
if [ "$INIT" = 1 ]; then I15="--init checkpoints/gnn_bg2_z32_i15_h64.pt"; I10="--init checkpoints/gnn_bg2_z32_i10_h64.pt"; fi
timeout -k 10 $((M15 * 60 + 240)) python -u tools/train_gnn_checkpoint.py --layers 15 --minutes $M15 $I15 \
  --out $C/gnn_bg2_z32_i15_h64.pt > $O/train_i15.log 2>&1 || { tail -20 $O/train_i15.log; exit 1; }
tail -2 $O/train_i15.log
timeout -k 10 $((M10 * 60 + 240)) python -u tools/train_gnn_checkpoint.py --layers 10 --minutes $M10 $I10 \
  --out $C/gnn_bg2_z32_i10_h64.pt > $O/train_i10.log 2>&1 || { tail -20 $O/train_i10.log; exit 1; }
tail -2 $O/train_i10.log
B="timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --steps 5 --warmup 1"
for d in zero codewords; do
  $B --data $d --workload gnn-z32-bf16 --checkpoint $C/gnn_bg2_z32_i15_h64.pt > $O/gnn_z32_bf16_$d.json || exit 1
  $B --data $d --workload gnn-z32 --checkpoint $C/gnn_bg2_z32_i10_h64.pt > $O/gnn_z32_$d.json || exit 1
  for s in 1 3 4; do
    $B --data $d --workload gnn-z32-bf16 --snr $s --checkpoint $C/gnn_bg2_z32_i15_h64.pt > $O/gnn_z32_bf16_${d}_snr$s.json || exit 1
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), 'cw/s', 'ber', d['ber'], 'fer', d['fer'], 'avg_layers', d['avg_layers'])"; done
