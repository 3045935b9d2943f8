#!/bin/bash
# GPU call: fp6 feed probe (+ DMA-only), projection engines incl. the ping-pong forms.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03d}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 300 python -u tools/bench_proj.py --engines i8,pp4,pp5,s5 > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.err; ok $?
cut -c1-900 gpurun_out/${T}_proj.json; tail -3 gpurun_out/${T}_proj.err
FEEDTEST=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_feedtest.log 2>&1; ok $?
cat gpurun_out/${T}_feedtest.log
