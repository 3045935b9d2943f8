#!/bin/bash
# GPU call: fp6 feed probe, projection engines, chi-square suite + profile, rank-share probes.
# Stops at the first fault / abort / timeout.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03c}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
FEEDTEST=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_feedtest.log 2>&1; ok $?
cat gpurun_out/${T}_feedtest.log
timeout -k 10 300 python -u tools/bench_proj.py > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.err; ok $?
cut -c1-600 gpurun_out/${T}_proj.json
for G in 8 4 1; do
  timeout -k 10 300 python -u tools/probe_rank_share.py --gpus $G > gpurun_out/${T}_rank_share_$G.json 2> gpurun_out/${T}_rank_share_$G.err; ok $?
  cat gpurun_out/${T}_rank_share_$G.json
done
bash tools/gpu_chi2.sh ${T}_chi2
