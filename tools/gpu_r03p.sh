# Round 3: kernel breakdown of cfg5 with early termination (random codewords), stamped PMC of BP Z=32
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r03p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_cfg5 -o run -- python3 $R/bench.py --workload gnn-z32-bf16 --data codewords --steps 2 --warmup 1 --cpu-baseline-seconds 0 > $R/$O/prof_cfg5.log 2>&1 || exit 1
echo cfg5 prof ok
cd $R && bash tools/gpu_profile.sh bp-z32 r03p || exit 1
