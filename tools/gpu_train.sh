#!/bin/bash
# GPU call: training regime tests, the configs[4] training bench at full scale, and its rocprofv3
# kernel trace (stats) -- run from the repo root on the GPU box.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/prof_train
T=${1:-r02d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -k "${KSEL:-regimes or sharded_training or eigh or sygv or fisherfaces}" -v --timeout 250 \
    --timeout-method thread > gpurun_out/${T}_train_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_train_tests.txt
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u tools/bench_train.py --n 100000 --ids 10000 --solver ${SOLVER:-auto} \
    > gpurun_out/${T}_train_full.json 2> gpurun_out/${T}_train_full.log || exit $?
cut -c1-900 gpurun_out/${T}_train_full.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_train -o kt \
    -- python3 $R/tools/bench_train.py --n 100000 --ids 10000 --solver ${SOLVER:-auto} --n-cpu 100 \
    > $R/gpurun_out/prof_train/kt.log 2>&1 || exit $?
head -12 $R/gpurun_out/prof_train/kt_kernel_stats.csv
exit $rc
