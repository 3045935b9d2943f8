cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2; do for o in 1 0; do
OFR_BENCH_OVERLAP=$o timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu --small-batches "" --stress "" --config1 0 > gpurun_out/ab_${o}_${r}.json 2>/dev/null || exit $?
python -c "import json;r=json.loads(open('gpurun_out/ab_${o}_${r}.json').read().strip().splitlines()[-1]);print('overlap=$o', round(r['value']), round(r['ms_per_step'],3), {k:round(v,3) for k,v in r['kernels_ms'].items()})"
done; done
