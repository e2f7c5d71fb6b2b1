# Profile one bench workload: kernel trace + stats, then PMC counters in separate passes
# (never combined with other tracing -- see the MI355X profiling rules).
# usage: bash tools/gpu_profile.sh <workload> <tag> [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
W=${1:-minsum-z32}; TAG=${2:-r01}; shift 2; EXTRA="$@"
OUT=$R/gpurun_out/prof_${TAG}_${W}
mkdir -p $OUT
# stamp: the library build these counters describe (bench.py refuses PMC figures of another build)
sha256sum ${LDPC_AMD_LIB:-$R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so} > $OUT/lib_sha256.txt || exit 1
# and of each of its gfx950 code objects (bench.py also accepts a stamp on the benched kernel's one)
python3 $R/tools/code_object_sha.py --all ${LDPC_AMD_LIB:-$R/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/libldpc_amd.so} > $OUT/code_objects_sha256.txt || exit 1
cd /tmp && export TMPDIR=/tmp
ok() { rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload $W --steps 10 --warmup 2 --cpu-baseline-seconds 0 $EXTRA > $OUT/trace_bench.log 2>&1; ok $?; echo "trace rc=$rc"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc1 -o run -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --cpu-baseline-seconds 0 $EXTRA > $OUT/pmc1.log 2>&1; ok $?; echo "pmc1 rc=$rc"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --cpu-baseline-seconds 0 $EXTRA > $OUT/pmc2.log 2>&1; ok $?; echo "pmc2 rc=$rc"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --cpu-baseline-seconds 0 $EXTRA > $OUT/pmc3.log 2>&1; ok $?; echo "pmc3 rc=$rc"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc4 -o run -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --cpu-baseline-seconds 0 $EXTRA > $OUT/pmc4.log 2>&1; ok $?; echo "pmc4 rc=$rc"
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc5 -o run -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --cpu-baseline-seconds 0 $EXTRA > $OUT/pmc5.log 2>&1; ok $?; echo "pmc5 rc=$rc"
ls -R $OUT | head -50
