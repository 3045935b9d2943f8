# round 6: the merge's deep continuation: the whole -m gpu suite, then the bench with stress (deep on, then off)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06am}
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -15 gpurun_out/${T}_gpu_tests.txt | grep -E "passed|failed|FAILED|Error" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in 1 0; do
OFR_MERGE_DEEP=$m timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.log || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_bench_$m.json').read())
print('deep $m', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], d['uncertified_after_each_tier'])
for s in d['stress']: print('   stress', s['pixel_noise'], round(s['queries_per_s']), s['uncertified_after_each_tier'], s['fallback_ms_per_step'], s['top1_identity_acc'])"
done
exit $rc
