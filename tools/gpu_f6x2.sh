#!/bin/bash
# GPU call for the two-slice fp6 tier: its parity tests and the routing / fallback tests, then the
# stress bench (crowded galleries, where the fp6 tier fails and f6x2 takes over).
# Stops at the first fault / abort / timeout (exit status other than 0 or 1).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r02_f6x2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "${KSEL:-f6x2 or routing or forces_fallback or append or overflow or euclidean_paths or f6_quantize}" \
    -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
[ "${BENCH:-1}" = "1" ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --no-cpu --small-batches "" --config1 0 \
    --stress "${STRESS:-48,96,192}" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
tail -4 gpurun_out/${T}_bench.log
exit $rc
