# round 6: the deep continuation as a second launch (merge_kernel<.., DEEP>): tests, bench with stress
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06as}
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "crowded or deep_merge or resieve or adaptive or prefix or sieve or pipeline or headline or shard" > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.txt | grep -E "passed|failed"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${T}_tests.txt | head; exit $rc; fi
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_bench.json').read())
print(round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline_merge']['ms_alone'], d['uncertified_after_each_tier'])
for s in d['stress']: print('   stress', s['pixel_noise'], round(s['queries_per_s']), s.get('start_tiers'), s['uncertified_after_each_tier'], s['fallback_ms_per_step'])"
