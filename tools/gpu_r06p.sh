# round 6: the wave-decoupled prefix pass (engine 4) -- probe A/B against engine 3, the prefix tests under it, bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06p}
timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 4,3,4,3 --tag in-tree > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }
cat gpurun_out/${T}_probe.jsonl
OFR_F6P_ENGINE=4 timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 800 --timeout-method thread -k "prefix or sieve or shard or sharded or headline or config1" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for e in 4 3; do
OFR_F6P_ENGINE=$e timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$e.json 2> gpurun_out/${T}_bench_$e.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$e.json').read());print('engine $e', round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
done
exit $rc
