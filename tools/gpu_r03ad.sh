# Round 3: a fourth deep-supervision fine-tune stage of the 15-layer checkpoint; cfg5 lines from it
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03ad; mkdir -p $O gpurun_out/ckpt4
timeout -k 10 1000 python3 -u tools/train_gnn_checkpoint.py --layers 15 --minutes ${TRAIN_MIN:-15} --layer-loss all --lr 2e-4 \
  --seed 4 --init checkpoints/gnn_bg2_z32_i15_h64.pt --out gpurun_out/ckpt4/gnn_bg2_z32_i15_h64.pt > $O/train_i15.log 2>&1 || { tail -20 $O/train_i15.log; exit 1; }
tail -2 $O/train_i15.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'), 'fer', d.get('fer'), 'L', d.get('avg_layers'))"
}
CK="--checkpoint gpurun_out/ckpt4/gnn_bg2_z32_i15_h64.pt"
run cw_new --workload gnn-z32-bf16 --data codewords $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
run cw_prev --workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
run zero_new --workload gnn-z32-bf16 $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
run cw_new_snr1 --workload gnn-z32-bf16 --data codewords --snr 1 $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
