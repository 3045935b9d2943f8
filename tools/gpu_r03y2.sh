#!/bin/bash
# Round-3 GPU call: the wide sieve engine of earlier commits (tools/var/libw<commit>.so, built from
# those commits' csrc) against HEAD's -- the identical-row sieve probe (34,000 rows must be kept)
# and the bench's sieve pass.  Stops at the first failed step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03y2}
A="--steps 10 --warmup 2 --stress= --small-batches= --no-cpu --config1 0"
for m in ${VARIANTS:-head w580fa09}; do
  L=""; [ $m = head ] || L="OFR_LIB=$R/tools/var/lib$m.so"
  env $L timeout -k 10 120 python -u tools/probe_sieve_dups.py > gpurun_out/${T}_${m}_dups.json 2>&1 || exit $?
  echo $m dups $(tail -1 gpurun_out/${T}_${m}_dups.json | cut -c1-120)
  env $L timeout -k 10 300 python -u bench.py $A > gpurun_out/${T}_${m}.json 2> gpurun_out/${T}_${m}.err || exit $?
  python - gpurun_out/${T}_${m}.json $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value", round(d["value"]), "ms", round(d["ms_per_step"], 3), "sieve_ms", round(d["roofline"]["launch_ms"], 3),
      "frac", round(d["roofline"]["frac"], 4), "uncert", d["uncertified_queries_per_step"], "acc", d["top1_identity_acc"])
PY
done
