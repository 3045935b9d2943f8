#!/bin/bash
# GPU call: chi-square tests (MFMA and VALU passes, LBPH model), configs[3] bench through both
# engines and the model API, rocprofv3 kernel stats of the bench.  Stops at a fault / abort / timeout.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/prof_chi2
T=${1:-r03_chi2}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_lbph_model.py tests/test_gpu_shard_api.py -k "chi2 or lbph or Chi" > gpurun_out/${T}_tests.txt 2>&1; ok $?
grep -E "passed|failed" gpurun_out/${T}_tests.txt | tail -3
timeout -k 10 400 python -u tools/bench_lbp_chi2.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; ok $?
cut -c1-1200 gpurun_out/${T}_bench.json
OFR_CHI2_ENGINE=valu timeout -k 10 400 python -u tools/bench_lbp_chi2.py --cpu-seconds 1 > gpurun_out/${T}_bench_valu.json 2>&1; ok $?
timeout -k 10 400 python -u tools/bench_lbph_model.py > gpurun_out/${T}_model.json 2> gpurun_out/${T}_model.err; ok $?
cut -c1-800 gpurun_out/${T}_model.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_chi2 -o kt \
    -- python3 $R/tools/bench_lbp_chi2.py --cpu-seconds 1 > $R/gpurun_out/prof_chi2/run.log 2>&1; ok $?
head -8 $R/gpurun_out/prof_chi2/kt_kernel_stats.csv | cut -c1-220
