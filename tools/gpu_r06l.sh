# round 6: the projection with the images straight to VGPRs (bd) against the LDS-staged engine (blds):
# bit-identical outputs and times, twice; then the projection tests and a short bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06l}
timeout -k 10 300 python -u tools/bench_proj.py --engines bd,blds,bd,blds > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.log || { cat gpurun_out/${T}_proj.log | tail -20; exit 1; }
cat gpurun_out/${T}_proj.json
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -k "projection or project or parity or test_gpu_prefix" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read());print(round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
exit $rc
