#!/bin/bash
# GPU call: the whole -m gpu suite, smoke, the default bench line, then the 8-rank rehearsal.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03p}
BENCH_ARGS="--steps 10 --warmup 2" TEST_TIMEOUT=700 BENCH_TIMEOUT=500 bash tools/gpu_round.sh $T || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
bash tools/gpu_rehearse_ranks.sh 8
