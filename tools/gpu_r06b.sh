# round 6: the two-workgroups-per-CU prefix pass -- parity tests, then a same-box A/B of the bench
# against the round-5 engine (OFR_F6P_ENGINE=1), then a kernel trace of the new pass
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06b}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -k "prefix or sieve or headline or pipeline or config1" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for e in 2 1 2 1; do
  OFR_F6P_ENGINE=$e timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_e$e.json 2> gpurun_out/${T}_bench_e$e.log || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_e$e.json').read());print('engine $e', round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 || exit $?
echo prof ok
