# Round 3: fine-tune the 10-layer Z=32 checkpoint (the reference's last-layer loss); cfg4 lines from it
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03ag; mkdir -p $O gpurun_out/ckpt10
timeout -k 10 900 python3 -u tools/train_gnn_checkpoint.py --layers 10 --minutes ${TRAIN_MIN:-12} --layer-loss last --lr 5e-4 \
  --seed 5 --init checkpoints/gnn_bg2_z32_i10_h64.pt --out gpurun_out/ckpt10/gnn_bg2_z32_i10_h64.pt > $O/train_i10.log 2>&1 || { tail -20 $O/train_i10.log; exit 1; }
tail -2 $O/train_i10.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'), 'fer', d.get('fer'))"
}
CK="--checkpoint gpurun_out/ckpt10/gnn_bg2_z32_i10_h64.pt"
run cw_new --workload gnn-z32 --data codewords $CK --steps 2 --warmup 1 --cpu-baseline-seconds 0
run cw_prev --workload gnn-z32 --data codewords --steps 2 --warmup 1 --cpu-baseline-seconds 0
run bf16_cw_new --workload gnn-z32-bf16-i10 --data codewords $CK --steps 2 --warmup 1 --cpu-baseline-seconds 0
