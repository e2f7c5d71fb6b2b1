# Round-3 final evidence (final checkpoints and grid cap): smoke, every GPU test, every bench line (gpurun_out/bench_all), fp32 GNN HBM bytes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_all.sh || exit $?
O=$R/gpurun_out/pmc_gnn_z32; mkdir -p $O
sha256sum $R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so > $O/lib_sha256.txt
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --workload gnn-z32 --batch 10923 --steps 1 --warmup 1 --cpu-baseline-seconds 0"
LDPC_GNN_STREAMS=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc3 -o run -- $B > $O/pmc3.log 2>&1 || exit 1
LDPC_GNN_STREAMS=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4 -o run -- $B > $O/pmc4.log 2>&1 || exit 1
echo pmc ok
