#!/bin/bash
# Round-3 GPU call K: the training determinism diagnostic, the ingest test file, smoke, then the
# rocprofv3 kernel trace + PMC passes of the search pass.  Stops at the first failed step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03k}
REPS=24 timeout -k 10 300 python -u tools/diag_train_nan.py > gpurun_out/${T}_diag_train_nan.jsonl 2>&1 || exit $?
tail -1 gpurun_out/${T}_diag_train_nan.jsonl
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ingest.py > gpurun_out/${T}_ingest_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/${T}_ingest_tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
bash tools/prof_search.sh || exit $?
echo prof done
