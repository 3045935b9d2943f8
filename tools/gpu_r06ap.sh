# round 6: the deep continuation's round cap on the stress galleries (32, the default, vs 256) + the deep test
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ap}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "crowded or deep_merge" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for m in 256 32; do
OFR_MERGE_DEEP=$m timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.log || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_bench_$m.json').read())
print('deep $m', round(d['value']), round(d['ms_per_step'],3), d['uncertified_after_each_tier'])
for s in d['stress']: print('   stress', s['pixel_noise'], round(s['queries_per_s']), s['uncertified_after_each_tier'], s['fallback_ms_per_step'])"
done
