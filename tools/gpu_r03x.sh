#!/bin/bash
# Round-3: pipeline + search GPU tests on the default (wide) engine, then the bench line.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03x}
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -k "${KSEL:-pipeline or knn or f6 or adaptive}" \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; ok $?
tail -3 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches "" \
    > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log; ok $?
cut -c1-300 gpurun_out/${T}_bench.json
