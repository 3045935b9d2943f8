# round 6: the projection as two tile-range launches with the previous batch's merge beside the last round
# (bench merge_at "tail") vs "after": tests, then the default bench alternating both schedules
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ay}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "tile_ranges or step_pipeline" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for st in after tail after tail; do
OFR_BENCH_MERGE=$st timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$st.json 2> gpurun_out/${T}_bench_$st.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$st.json').read());print('$st', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, d['uncertified_after_each_tier'], d['top1_identity_acc'])"
done
