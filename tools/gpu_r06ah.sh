# round 6: bench step schedule A/B: merge behind the tile pass ("after") vs beside the next sample pass ("sample")
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ah}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for m in sample after sample after; do
OFR_BENCH_MERGE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$m.json 2> gpurun_out/${T}_bench_$m.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$m.json').read());print('$m', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], d['uncertified_after_each_tier'])"
done
