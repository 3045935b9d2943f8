#!/bin/bash
# The whole GPU suite + smoke on the current tree.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03s}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/${T}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1; rc=$?
tail -2 gpurun_out/${T}_smoke.txt; exit $rc
