#!/bin/bash
# GPU call: pipeline + adaptive-start tests, the fallback/tier parity tests, then the bench line.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03r}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -v -s --timeout 240 --timeout-method thread -m gpu -k "pipeline or adaptive or fallback or f6x2 or f6_tier or sieve or crowded or knn" > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -30 gpurun_out/${T}_bench.log; exit 1; }
python - <<PY
import json; r=json.load(open("gpurun_out/${T}_bench.json"))
print(r["value"], r["ms_per_step"], r["kernels_ms"], r["start_tiers"], r["config1"]["queries_per_s"])
for s in r.get("stress", []): print(s["pixel_noise"], s["queries_per_s"], s["start_tiers"], s["uncertified_after_each_tier"], s["fallback_ms_per_step"], s["top1_identity_acc"])
PY
