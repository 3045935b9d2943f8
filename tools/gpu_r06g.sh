# round 6: merge placement (after the tile pass vs under the sieve pass) x prefix-pass engine, same box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
for cfg in after:2 sieve:2 after:1 sieve:1 after:2 after:1; do
  m=${cfg%%:*}; e=${cfg##*:}
  OFR_BENCH_MERGE=$m OFR_F6P_ENGINE=$e timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_${m}_$e.json 2> gpurun_out/${T}_bench_${m}_$e.log || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_${m}_$e.json').read());print('merge $m engine $e', round(d['value']), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms'].items()}, round(d['roofline']['launch_ms'],3), d['uncertified_after_each_tier'])"
done
