#!/bin/bash
# Round-3 wide-engine evidence: bench line (default engine), then rocprofv3 stats + PMC passes of the
# search kernels (tools/prof_search.sh).  Stops at the first fault / timeout.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03w}
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches "" \
    > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log; ok $?
cut -c1-300 gpurun_out/${T}_bench.json
[ -n "$NO_PROF" ] && exit 0
bash tools/prof_search.sh; ok $?
grep -E "tile_kernel|sieve|merge|project|quantize" gpurun_out/prof/kt/*kernel_stats.csv | cut -c1-250
