# Two SQ counter passes (stall breakdown + MFMA busy) of one bench workload, one stream, for the
# default library and variant libraries (ab/<name>.so): gpurun_out/pmcab_<TAG>/<lib>/p{1,2}.
# BYTES=1 adds FETCH_SIZE / WRITE_SIZE passes (p3, p4).
# usage: TAG=x bash tools/gpu_pmc_ab.sh "<variant names>" [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmcab_${TAG:-x}; mkdir -p $O
VARS=$1; shift
pass() {  # lib-tag lib pass counters...
  local t=$1 lib=$2 p=$3; shift 3
  LDPC_GNN_STREAMS=1 LDPC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$t/$p -o run -- python3 $R/bench.py --cpu-baseline-seconds 0 --steps 1 --warmup 1 $ARGS > $O/$t/$p.log 2>&1 || { echo "$t $p rc=$?"; exit 1; }
  echo "$t $p ok"
}
ARGS="$@"
for v in base $VARS; do
  lib=$R/ab/$v.so; [ $v = base ] && lib=$R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so
  mkdir -p $O/$v
  pass $v $lib p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
  pass $v $lib p2 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM
  if [ -n "$BYTES" ]; then pass $v $lib p3 FETCH_SIZE; pass $v $lib p4 WRITE_SIZE; fi
done
