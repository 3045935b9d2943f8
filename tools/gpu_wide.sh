#!/bin/bash
# GPU call for the wide fp6 sieve engine (f6t::EngineW, OFR_F6_SHAPE=384): probe timings against the
# library pass, the search parity tests on the wide engine, a bench line.  Stops at the first fault.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03w}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
WIDE=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_probe.log 2>&1; ok $?
cat gpurun_out/${T}_probe.log
[ -n "$PROBE_ONLY" ] && exit 0
OFR_F6_SHAPE=384 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "${KSEL:-knn or f6}" -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; ok $?
tail -3 gpurun_out/${T}_tests.txt
OFR_F6_SHAPE=384 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches "" \
    > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log; ok $?
cut -c1-600 gpurun_out/${T}_bench.json
