#!/bin/bash
# GPU call: fp6 feed probes (library kernel variants, then the pure copy probe).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03h}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
FEEDTEST=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_feedtest.log 2>&1; ok $?
cat gpurun_out/${T}_feedtest.log
timeout -k 10 200 ./tools/feed_probe 1000000 4096 9999 3 > gpurun_out/${T}_feed.log 2>&1; ok $?
cat gpurun_out/${T}_feed.log
