# round 6 (re-entry): the whole GPU suite, smoke, the default bench and a kernel trace of the bench on HEAD
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06e}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -2 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read());print(round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['roofline']['frac'], d['uncertified_after_each_tier'], d.get('roofline_merge'))"
exit $rc
