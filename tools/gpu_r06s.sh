# round 6: block-cooperative merge re-rank (default) vs the wave form (OFR_MERGE_ENGINE=1): GPU tests, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06s}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "prefix or sieve or shard or sharded or headline or config1 or pipeline or deep_k or parity or merge" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for e in 2 1 2 1; do
OFR_MERGE_ENGINE=$e timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$e.json 2> gpurun_out/${T}_bench_$e.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$e.json').read());m=d['roofline_merge'];print('merge engine $e', round(d['value']), round(d['ms_per_step'],3), d['kernels_ms'], 'merge alone', round(m['ms_alone'],3), 'evals', round(m['exact_reranks_per_query'],2), 'frac', round(m['frac'],3), d['uncertified_after_each_tier'])"
done
exit $rc
