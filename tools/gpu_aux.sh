#!/bin/bash
# GPU call: training GEMM / Gram and LBP / chi-square -- tests, throughput tools and rocprofv3
# kernel-trace summaries.  Stops at the first fault / abort / timeout.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/prof_aux
T=${1:-r02h}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
    -k "${KSEL:-gemm or regimes or fisherfaces or chi2 or lbp or spatial or sharded_training}" -q --timeout 300 \
    --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; ok $?
tail -3 gpurun_out/${T}_tests.txt
if [ -z "${SKIP_GEMM:-}" ]; then
timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/${T}_gemm.json 2>&1; ok $?
cat gpurun_out/${T}_gemm.json
fi
timeout -k 10 400 python -u tools/bench_lbp_chi2.py > gpurun_out/${T}_lbp_chi2.json 2> gpurun_out/${T}_lbp_chi2.err; ok $?
cut -c1-1500 gpurun_out/${T}_lbp_chi2.json
cd /tmp && export TMPDIR=/tmp
if [ -z "${SKIP_GEMM:-}" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_aux/gemm -o kt \
    -- python3 $R/tools/bench_gemm.py > $R/gpurun_out/prof_aux/gemm.log 2>&1; ok $?
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_aux/lbp -o kt \
    -- python3 $R/tools/bench_lbp_chi2.py --cpu-seconds 1 > $R/gpurun_out/prof_aux/lbp.log 2>&1; ok $?
[ -z "${SKIP_GEMM:-}" ] && head -6 $R/gpurun_out/prof_aux/gemm/kt_kernel_stats.csv | cut -c1-200
head -8 $R/gpurun_out/prof_aux/lbp/kt_kernel_stats.csv | cut -c1-200
