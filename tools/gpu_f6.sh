#!/bin/bash
# GPU call for the fp6 engine: probe, parity tests of the search, benches (16x16 and 32x32 sieve).
# Stops at the first fault / abort / timeout (exit status other than 0 or 1).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r02f}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
SHAPE16=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_shape16.log 2>&1; ok $?
cat gpurun_out/${T}_shape16.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "${KSEL:-knn or f6 or projection}" -q --timeout 300 \
    --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; ok $?
tail -3 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches 1 \
    > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log; ok $?
cut -c1-400 gpurun_out/${T}_bench.json
OFR_F6_SHAPE=32 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches "" \
    > gpurun_out/${T}_bench32.json 2> gpurun_out/${T}_bench32.log; ok $?
cut -c1-400 gpurun_out/${T}_bench32.json
