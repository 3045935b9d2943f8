# round 6: the fp6 tier's second sieve pass for open queries: its tests, the crowded/deep tests, then the stress bench (on/off)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06aq}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -q -s --timeout 300 --timeout-method thread -k "crowded or deep_merge or resieve or adaptive" > gpurun_out/${T}_tests.txt 2>&1
rc=$?
grep -E "open after|passed|failed|FAILED|Error" gpurun_out/${T}_tests.txt | head -20
if [ $rc -ne 0 ]; then tail -40 gpurun_out/${T}_tests.txt; exit $rc; fi
for m in 1 0; do
OFR_RESIEVE=$m timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.log || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_bench_$m.json').read())
print('resieve $m', round(d['value']), round(d['ms_per_step'],3), d['uncertified_after_each_tier'])
for s in d['stress']: print('   stress', s['pixel_noise'], round(s['queries_per_s']), round(s['ms_per_step'],2), s['uncertified_after_each_tier'], s['fallback_ms_per_step'], s['top1_identity_acc'])"
done
