#!/bin/bash
# Round-3 evidence on the final engines: whole GPU suite + smoke, bench (default flags), rocprofv3 stats +
# PMC of the search kernels.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03f}
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
[ -z "$NO_SUITE" ] && { bash tools/gpu_suite.sh ${T}; ok $?; }
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log; ok $?
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('phase1'), d['kernels_ms'], d.get('config1', {}).get('queries_per_s'))"
[ -n "$NO_PROF" ] && exit 0
bash tools/prof_search.sh "tile_kernel_f6|sieve_threshold|project_q8w"; ok $?
grep -E "tile_kernel|sieve|merge|project|quantize" gpurun_out/prof/kt/*kernel_stats.csv | cut -c1-200
