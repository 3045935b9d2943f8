# round 6: prefix pass without the spurious vmcnt waits, the wave-parallel merge sort -- probe, tests, bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06d}
timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 2,1 --tag in-tree > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || exit $?
cat gpurun_out/${T}_probe.jsonl
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -k "prefix or sieve or headline or shard or sharded or pipeline or knn or chi2 or deep or merge or lbph" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read());print(round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'], d.get('roofline_merge'), d.get('brute_force_equivalent'))"
