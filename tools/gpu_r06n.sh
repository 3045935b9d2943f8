# round 6: the compact hit path of the folded prefix pass -- probe, prefix tests, bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06n}
timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 3,2,3 --tag in-tree > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }
cat gpurun_out/${T}_probe.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 800 --timeout-method thread -k "prefix or sieve or shard or sharded or headline or config1" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read());print(round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
exit $rc
