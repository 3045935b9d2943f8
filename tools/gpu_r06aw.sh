# round 6: register-staged stage copies of the exact projection (OFR_PROJ_STAGE=reg) vs LDS-DMA: bit identity,
# timing at the bench shape, the projection tests on the reg form, then the bench both ways
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06aw}
timeout -k 10 300 python -u tools/bench_proj.py --engines dma,reg,dma,reg > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.log || { tail -30 gpurun_out/${T}_proj.log; cat gpurun_out/${T}_proj.json; exit 1; }
cat gpurun_out/${T}_proj.json
OFR_PROJ_STAGE=reg timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "project or config1 or ctx_abi" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for st in dma reg; do
OFR_PROJ_STAGE=$st timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_$st.json 2> gpurun_out/${T}_bench_$st.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$st.json').read());print('$st', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, d['uncertified_after_each_tier'])"
done
