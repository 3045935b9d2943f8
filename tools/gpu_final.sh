#!/bin/bash
# Round-end evidence in one GPU call: the whole -m gpu suite + smoke + the default bench line,
# then the rocprofv3 kernel trace and PMC passes of the search pass (tools/prof_search.sh).
# Stops at the first step that faults, aborts or times out.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02_final}
BENCH_ARGS="${BENCH_ARGS:-}" TEST_TIMEOUT=700 BENCH_TIMEOUT=500 bash tools/gpu_round.sh $TAG || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || exit $?
[ "${PROF:-1}" = "1" ] || exit 0
bash tools/prof_search.sh ${PROF_K:-} || exit $?
echo "prof done: run python tools/pmc_summary.py $TAG locally after the merge"
