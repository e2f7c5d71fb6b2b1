# Round 3: deep-supervision fine-tune of the 15-layer Z=32 checkpoint (so cfg5's early termination
# fires), cfg5 bench lines from it (ET on / off, random codewords and all-zero), stamped min-sum PMC.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03h; mkdir -p $O gpurun_out/ckpt
timeout -k 10 480 python3 -u tools/train_gnn_checkpoint.py --layers 15 --minutes ${TRAIN_MIN:-6} --layer-loss all \
  --init checkpoints/gnn_bg2_z32_i15_h64.pt --out gpurun_out/ckpt/gnn_bg2_z32_i15_h64.pt > $O/train_i15.log 2>&1 || { tail -20 $O/train_i15.log; exit 1; }
tail -2 $O/train_i15.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { rc=$?; echo "bench $n rc=$rc"; tail -5 $O/$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); r=d['roofline']; print('$n', round(d['value']), 'frac', r['frac'], 'kern_ms', round(r['kernel_ms'],3), 'ber', d.get('ber'), 'fer', d.get('fer'), 'avg_layers', d.get('avg_layers'))"
}
CK="--checkpoint gpurun_out/ckpt/gnn_bg2_z32_i15_h64.pt"
run cfg5_cw --workload gnn-z32-bf16 --data codewords $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
run cfg5_zero --workload gnn-z32-bf16 $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
run cfg5_cw_noet --workload gnn-z32-bf16 --data codewords --early-termination off $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
for snr in 1 3; do
  run cfg5_cw_snr$snr --workload gnn-z32-bf16 --data codewords --snr $snr $CK --steps 3 --warmup 1 --cpu-baseline-seconds 0
done
bash tools/gpu_profile.sh minsum-z32 r03h || exit 1
