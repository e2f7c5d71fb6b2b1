# Round 3: longer deep-supervision fine-tune of the 15-layer checkpoint; cfg5 lines from it
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03aa; mkdir -p $O gpurun_out/ckpt2
# dW2 on bf16x6 splits (train_outer_split_kernel): gradient tests, then A/B against the fp32 kernel
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for sp in 1 0 1 0; do
  LDPC_GNN_OUTER_SPLIT=$sp timeout -k 10 120 python3 bench.py --workload gnn-train-z32 --steps 10 --warmup 2 --cpu-baseline-seconds 0 > $O/train_split$sp.json 2> $O/train.err || exit 1
  python3 -c "import json; d=json.load(open('$O/train_split$sp.json')); print('train split=$sp', round(d['value']), round(d['ms_per_step'],2))"
done
timeout -k 10 840 python3 -u tools/train_gnn_checkpoint.py --layers 15 --minutes ${TRAIN_MIN:-12} --layer-loss all --lr 5e-4 \
  --seed 2 --init checkpoints/gnn_bg2_z32_i15_h64.pt --out gpurun_out/ckpt2/gnn_bg2_z32_i15_h64.pt > $O/train_i15.log 2>&1 || { tail -20 $O/train_i15.log; exit 1; }
tail -2 $O/train_i15.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'), 'fer', d.get('fer'), 'L', d.get('avg_layers'))"
}
CK="--checkpoint gpurun_out/ckpt2/gnn_bg2_z32_i15_h64.pt"
run cw_new --workload gnn-z32-bf16 --data codewords $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
run zero_new --workload gnn-z32-bf16 $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
run cw_old --workload gnn-z32-bf16 --data codewords --steps 3 --warmup 1 --cpu-baseline-seconds 0
for snr in 1 3; do run cw_new_snr$snr --workload gnn-z32-bf16 --data codewords --snr $snr $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0; done
