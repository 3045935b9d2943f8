#!/bin/bash
# One GPU call: the -m gpu suite (minus the listed -k filter), then a short bench if the suite
# ended normally (0 = pass, 1 = test failures); any fault / abort / timeout stops the call.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r02}
KSEL=${2:-}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
    ${KSEL:+-k "$KSEL"} > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2} \
      > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
  brc=$?
  tail -3 gpurun_out/${TAG}_bench.log; cut -c1-600 gpurun_out/${TAG}_bench.json
  [ $brc -ne 0 ] && exit $brc
fi
exit $rc
