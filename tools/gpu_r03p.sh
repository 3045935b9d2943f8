#!/bin/bash
# Round-3: projection engines (bit-identical check + timing), then the whole GPU suite + smoke.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03p}
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 300 python tools/bench_proj.py --engines ${ENGINES:-i8,w} > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.log; ok $?
cat gpurun_out/${T}_proj.json
[ -n "$NO_SUITE" ] && exit 0
bash tools/gpu_suite.sh ${T}
