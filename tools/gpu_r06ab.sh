# round 6: after the wave pass grouping rule: tests (prefix/sieve/shard), rank share at G = 1/2/4/8, bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or sieve or shard or pipeline" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
: > gpurun_out/${T}_rank_share.jsonl
for G in 1 2 4 8; do
timeout -k 10 300 python -u tools/probe_rank_share.py --gpus $G >> gpurun_out/${T}_rank_share.jsonl 2> gpurun_out/${T}_rank_share_$G.log || { tail -20 gpurun_out/${T}_rank_share_$G.log; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/${T}_rank_share.jsonl'):
    d=json.loads(l); print(d['gpus'], {k: round(v,3) for k,v in d.items() if k.endswith('_ms')})"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read());print(round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
