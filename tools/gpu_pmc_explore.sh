# Extra PMC passes for one bench workload: instruction cache, VALU/LDS/SALU cycle counters.
# usage: bash tools/gpu_pmc_explore.sh <workload> <tag> [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
W=${1:-minsum-z32}; TAG=${2:-r02}; shift 2; EXTRA="$@"
OUT=$R/gpurun_out/pmcx_${TAG}_${W}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ok() { rc=$1; if [ $rc -ne 0 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
B="python3 $R/bench.py --workload $W --steps 2 --warmup 1 --cpu-baseline-seconds 0 $EXTRA"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1; ok $?; echo p1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1; ok $?; echo p2 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1; ok $?; echo p3 ok
