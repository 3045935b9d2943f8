#!/bin/bash
# Round-3: wide-engine probe, the shard API tests (pruned merge), the bench line.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03y}
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
WIDE_DEPTH=1 timeout -k 10 100 ./tools/f6_probe 1000000 4096 9999 3 > gpurun_out/${T}_probe.log 2>&1; ok $?
cat gpurun_out/${T}_probe.log
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_shard_api.py} -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_tests.txt 2>&1; ok $?
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches "" \
    > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log; ok $?
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms'], d['config1']['queries_per_s'])"
