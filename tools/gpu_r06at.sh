# round 6: bench schedule A/B: merge s-1 beside preparation s+1 ("prep") vs before it ("after", default)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06at}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for m in prep after prep after; do
OFR_BENCH_MERGE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$m.json').read());print('$m', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, d['uncertified_after_each_tier'])"
done
