#!/bin/bash
# GPU call: projection engines (timing + bit-identity), projection parity tests, then the chi-square
# call (tools/gpu_chi2.sh).  Stops at the first fault / abort / timeout.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03b}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 300 python -u tools/bench_proj.py > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.err; ok $?
cat gpurun_out/${T}_proj.json | cut -c1-1500; tail -5 gpurun_out/${T}_proj.err
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "project or fisher or Fisher" \
    > gpurun_out/${T}_proj_tests.txt 2>&1; ok $?
grep -E "passed|failed" gpurun_out/${T}_proj_tests.txt | tail -3
bash tools/gpu_chi2.sh ${T}_chi2
