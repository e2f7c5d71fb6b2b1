# Round 3: PMC passes over the bf16 GNN (10 layers, B=8192, one stream) for the MLP / group-mean kernels
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03r; mkdir -p $O
sha256sum $R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so > $O/lib_sha256.txt
cd /tmp && export TMPDIR=/tmp
export LDPC_GNN_STREAMS=1
B="python3 $R/bench.py --workload gnn-z32-bf16-i10 --batch 8192 --steps 1 --warmup 1 --cpu-baseline-seconds 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || exit 1
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc1 -o run -- $B > $O/pmc1.log 2>&1 || exit 1
echo pmc1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- $B > $O/pmc2.log 2>&1 || exit 1
echo pmc2 ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc3 -o run -- $B > $O/pmc3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4 -o run -- $B > $O/pmc4.log 2>&1 || exit 1
echo pmc ok
