#!/bin/bash
# Same-box A/B of library builds on the headline bench (run on the GPU box from the repo root):
#   bash tools/ab_lib.sh TAG ROUNDS LIB_A LIB_B [...]   (LIB "-": the in-tree library)
# Each round runs the short headline bench once per library, alternating, and appends one line per run
# (lib, step ms, sieve-pass ms by its events, queries/s, uncertified) to gpurun_out/TAG_ab.txt.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/${TAG}_ab.txt
ARGS=${AB_ARGS:---steps 10 --warmup 2 --no-cpu --small-batches= --stress= --config1 0 --config3 0 --api 0 --config4 0}
for r in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    if [ "$L" = "-" ]; then unset OFR_LIB; else export OFR_LIB=$R/$L; fi
    timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/${TAG}_run.json 2> gpurun_out/${TAG}_run.log || exit $?
    python -c "
import json, sys
d = json.loads([l for l in open('gpurun_out/${TAG}_run.json') if l.startswith('{')][-1])
print('round', $r, 'lib', '$L', 'step_ms %.3f' % d['ms_per_step'], 'sieve_ms %.3f' % d['roofline']['launch_ms'],
      'qps %.0f' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'uncert', d['uncertified_after_each_tier'],
      'prep_ms %.3f' % list(d['kernels_ms'].values())[0])
" | tee -a $OUT
  done
done
