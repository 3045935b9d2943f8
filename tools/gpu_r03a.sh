#!/bin/bash
# Round-3 GPU call A: the new parity tests (LBPH model end to end, sharded API near-tie rule,
# full-size configs[2] on two gloo ranks, configs[4] default solver vs eigh, ctx ABI), then the
# LBPH model-API bench.  Stops at the first fault / abort / timeout.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03a}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -s -v --timeout 700 --timeout-method thread \
    ${TESTS:-tests/test_gpu_lbph_model.py tests/test_gpu_shard_api.py tests/test_gpu_ctx_abi.py tests/test_gpu_configs.py} \
    ${KSEL:+-k "$KSEL"} > gpurun_out/${T}_tests.txt 2>&1; ok $?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/${T}_tests.txt | tail -30
if [ "${BENCH_LBPH:-1}" = "1" ]; then
timeout -k 10 400 python -u tools/bench_lbph_model.py > gpurun_out/${T}_lbph_model.json 2> gpurun_out/${T}_lbph_model.err; ok $?
cut -c1-1500 gpurun_out/${T}_lbph_model.json
fi
