# round 6: the folded prefix pass after the rebuild -- prefix / sharded / shard-api tests, probe, bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06k}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 800 --timeout-method thread -k "prefix or sieve or shard or sharded or headline or config1 or pipeline" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/diag_shard_prefix.py > gpurun_out/${T}_diag.txt 2>&1 || exit $?
grep engine gpurun_out/${T}_diag.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read());print(round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
exit $rc
