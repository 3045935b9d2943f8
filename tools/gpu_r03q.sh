#!/bin/bash
# GPU call: the step-pipeline test, then the default bench line on the three-stage schedule.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v -s --timeout 240 --timeout-method thread -m gpu > gpurun_out/${T}_pipe_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_pipe_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_pipe_tests.txt
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -30 gpurun_out/${T}_bench.log; exit 1; }
python - <<PY
import json; r=json.load(open("gpurun_out/${T}_bench.json"))
print(r["value"], r["ms_per_step"], r["kernels_ms"], r["config1"]["queries_per_s"], r["config1"]["ms_per_step"])
for s in r.get("stress", []): print(s["pixel_noise"], s["queries_per_s"], s["uncertified_after_each_tier"])
PY
