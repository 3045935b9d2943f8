#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03i}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
FEED4W=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_feed4w.log 2>&1; ok $?
cat gpurun_out/${T}_feed4w.log
GGDMA=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_ggdma.log 2>&1; ok $?
cat gpurun_out/${T}_ggdma.log
