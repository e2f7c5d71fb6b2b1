# kernel-trace A/B: new lib vs ab/head.so on gnn-z32, interleaved twice
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/kt_projgen; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
 for v in base head; do
  lib=$R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so; [ $v = head ] && lib=$R/ab/head.so
  LDPC_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$r -o run -- python3 $R/bench.py --workload gnn-z32 --steps 10 --warmup 2 --cpu-baseline-seconds 0 > $O/${v}_$r.log 2>&1 || exit 1
  echo "== $v $r"; python3 $R/tools/trace_summary.py $O/${v}_$r | head -6
 done
done
