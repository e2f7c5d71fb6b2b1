# Round 3: stage 5 of the 15-layer Z=32 checkpoint (deep supervision, lr 1e-4); cfg5 lines new vs current
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03am; mkdir -p $O gpurun_out/ckpt5
timeout -k 10 1000 python3 -u tools/train_gnn_checkpoint.py --layers 15 --minutes ${TRAIN_MIN:-13} --lr 1e-4 \
  --seed 6 --init checkpoints/gnn_bg2_z32_i15_h64.pt --out gpurun_out/ckpt5/gnn_bg2_z32_i15_h64.pt > $O/train_i15.log 2>&1 || { tail -20 $O/train_i15.log; exit 1; }
tail -2 $O/train_i15.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']), 'L', d.get('avg_layers'), 'ber', d.get('ber'), 'fer', d.get('fer'))"
}
CK="--checkpoint gpurun_out/ckpt5/gnn_bg2_z32_i15_h64.pt"
A="--workload gnn-z32-bf16 --steps 3 --warmup 1 --cpu-baseline-seconds 0"
run cw_new $A --data codewords $CK
run cw_cur $A --data codewords
run zero_new $A $CK
run zero_cur $A
run cw_new_snr1 $A --data codewords --snr 1 $CK
run cw_cur_snr1 $A --data codewords --snr 1
