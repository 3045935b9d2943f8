# round 6: stress galleries started at f6 (OFR_ADAPTIVE_TIER=0) with the second sieve pass for up to 4096 open queries
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ar}
for cfg in "OFR_ADAPTIVE_TIER=0 OFR_RESIEVE_MAX=4096" "OFR_ADAPTIVE_TIER=0 OFR_RESIEVE_MAX=256"; do
env $cfg timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}.json 2> gpurun_out/${T}.log || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}.json').read())
print('$cfg', round(d['value']))
for s in d['stress']: print('   stress', s['pixel_noise'], round(s['queries_per_s']), round(s['ms_per_step'],2), s.get('start_tiers'), s['uncertified_after_each_tier'], s['fallback_ms_per_step'], s['top1_identity_acc'])"
done
