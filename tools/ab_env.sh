#!/bin/bash
# Same-box A/B of environment settings on the headline bench (run on the GPU box from the repo root):
#   bash tools/ab_env.sh TAG ROUNDS "VAR=a VAR2=b" "VAR=c" ...   ("-": no extra setting)
# Each round runs the short headline bench once per setting, alternating, and appends one line per run
# to gpurun_out/TAG_ab.txt.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/${TAG}_ab.txt
ARGS=${AB_ARGS:---steps 10 --warmup 2 --no-cpu --small-batches= --stress= --config1 0 --config3 0 --api 0 --config4 0}
for r in $(seq 1 $ROUNDS); do
  for S in "$@"; do
    if [ "$S" = "-" ]; then E=""; else E="$S"; fi
    env $E timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/${TAG}_run.json 2> gpurun_out/${TAG}_run.log || exit $?
    python -c "
import json
d = json.loads([l for l in open('gpurun_out/${TAG}_run.json') if l.startswith('{')][-1])
k = d['kernels_ms']
print('round', $r, 'env', '$S', 'step_ms %.3f' % d['ms_per_step'], 'sieve_ms %.3f' % d['roofline']['launch_ms'],
      'qps %.0f' % d['value'], 'uncert', d['uncertified_after_each_tier'],
      'prep_ms %.3f' % list(k.values())[0], 'merge_ms %.3f' % list(k.values())[2])
" | tee -a $OUT
  done
done
