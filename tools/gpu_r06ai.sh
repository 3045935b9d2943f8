# round 6: the prefix tier's sample pass as a wave pass (default) vs the tile pass (OFR_F6P_SAMPLE=tiles); tests; bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ai}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --tag g1_swave
OFR_F6P_SAMPLE=tiles run --tag g1_stiles
run --gallery 125000 --query-ids 100000 --tag g8_swave
OFR_F6P_SAMPLE=tiles run --gallery 125000 --query-ids 100000 --tag g8_stiles
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['pass_ms_median'],3), 'sample', round(d['sample_ms_median'],3), round(d['kept_mean'],1), d['kept_max'])"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or sieve or shard or headline or config1 or pipeline" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for m in wave tiles; do
OFR_F6P_SAMPLE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$m.json').read());print('$m', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], d['roofline']['phase1']['sample_ms'], d['uncertified_after_each_tier'], d['sieve_kept_rows_per_query'])"
done
