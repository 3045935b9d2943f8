#!/bin/bash
# GPU call: fp6 feed probe with an L2-resident feed and the tile-group sweep of the DMA alone.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03e}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
FEEDTEST=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_feedtest.log 2>&1; ok $?
cat gpurun_out/${T}_feedtest.log
GGDMA=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_ggdma.log 2>&1; ok $?
cat gpurun_out/${T}_ggdma.log
