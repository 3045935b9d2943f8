# round 6: merge_at "tail" with the projection's last round on a high-priority stream (OFR_BENCH_TAIL_HI=1) vs plain tail vs after
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06az}
for v in "tail 0" "tail 1" "after 0" "tail 0" "tail 1" "after 0"; do set -- $v
OFR_BENCH_MERGE=$1 OFR_BENCH_TAIL_HI=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_b.json 2> gpurun_out/${T}_b.log || { tail -20 gpurun_out/${T}_b.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_b.json').read());print('$1 hi=$2', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items() if v}, d['uncertified_after_each_tier'], d['top1_identity_acc'])"
done
