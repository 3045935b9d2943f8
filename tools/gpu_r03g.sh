#!/bin/bash
# Round-3 GPU call G: the wide sieve pass's tile grouping (OFR_F6W_GROUP gallery tiles per group)
# A/B on the headline bench, two alternating rounds.  Stops at the first failed step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03g}
A="--steps 10 --warmup 2 --stress= --small-batches= --no-cpu --config1 0"
for rep in 1 2; do
  for g in ${GROUPS_:-4 2 8 16}; do
    OFR_F6W_GROUP=$g timeout -k 10 300 python -u bench.py $A > gpurun_out/${T}_g${g}_${rep}.json 2> gpurun_out/${T}_g${g}_${rep}.err || exit $?
    python - gpurun_out/${T}_g${g}_${rep}.json $g <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("group", sys.argv[2], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "sieve_ms", round(d["roofline"]["launch_ms"], 3),
      "frac", round(d["roofline"]["frac"], 4), "uncert", d["uncertified_queries_per_step"], "acc", d["top1_identity_acc"])
PY
  done
done
