#!/bin/bash
# GPU call: the sharded / certificate / fallback GPU tests after the native pack / merge / kth / open-rows
# kernels replaced the torch glue, then 2- and 4-rank rehearsals of the sharded bench step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r03m}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "step rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_shard_api.py tests/test_gpu_parity.py \
   tests/test_gpu_configs.py -k "shard or fallback or cert or chi2 or sphere or overflow or merge or config2 or routing" \
   > gpurun_out/${T}_tests.txt 2>&1; ok $?
grep -E "passed|failed" gpurun_out/${T}_tests.txt | tail -3
bash tools/gpu_rehearse_ranks.sh 2 4
for S in 64 128 256; do
  OFR_SIEVE_STRIDE=$S timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --stress "" --small-batches "" --config1 0 \
     > gpurun_out/${T}_stride$S.json 2> gpurun_out/${T}_stride$S.log; ok $?
  python -c "import json;r=json.loads(open('gpurun_out/${T}_stride$S.json').read().strip().splitlines()[-1]);print($S, round(r['value']), round(r['ms_per_step'],3), r['kernels_ms'], r['uncertified_after_each_tier'], r['sieve_kept_rows_per_query'])"
done
