# round 6: bench after the 128 x 32 wave steps (two runs) + the prefix / sieve / shard tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ag}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or sieve or shard or pipeline or headline" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$r.json 2> gpurun_out/${T}_bench_$r.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$r.json').read());print(round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['phase1'], d['uncertified_after_each_tier'])"
done
