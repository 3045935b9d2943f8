#!/bin/bash
# Round-3 GPU call Z: the step schedule A/B -- batch s+1's preparation behind tile pass s (alone,
# OFR_BENCH_PREP=tiles) or behind sample pass s (under sieve pass s, OFR_BENCH_PREP=sample) --
# on the headline and configs[1], two alternating runs each; and the sieve pass of the previous
# commit's library (prev) and of one without the wide epilogue's sched barriers (v1).  Stops at the first failed step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03z}
A="--steps 10 --warmup 2 --stress= --small-batches= --no-cpu"
for rep in 1 2; do
  for m in tiles sample prev v1; do
    case $m in prev|v1) L="OFR_LIB=$R/tools/var/lib$m.so"; P=tiles;; *) L=""; P=$m;; esac
    env $L OFR_BENCH_PREP=$P timeout -k 10 300 python -u bench.py $A > gpurun_out/${T}_${m}_${rep}.json 2> gpurun_out/${T}_${m}_${rep}.err || exit $?
    python - gpurun_out/${T}_${m}_${rep}.json $m <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "config1", round(d["config1"]["queries_per_s"]),
      round(d["config1"]["ms_per_step"], 3), "sieve_frac", round(d["roofline"]["frac"], 4), d["kernels_ms"])
EOF
  done
done
