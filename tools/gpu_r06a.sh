set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 700 --timeout-method thread -k "projection or deep_k or headline or sieve_complete or config1 or prefix" > gpurun_out/r06a_gpu_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r06a_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --stress= --small-batches= --no-cpu > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.log
brc=$?
tail -3 gpurun_out/r06a_bench.log; cut -c1-1500 gpurun_out/r06a_bench.json
exit $rc
