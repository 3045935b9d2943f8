# round 6: prefix wave pass, grouping rule f6p_group_wave (items >= 6 per workgroup): G = 1/2/4/8 shards
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06x}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --tag g1
OFR_F6P_GROUP=64 run --tag g1_group64
run --gallery 500000 --query-ids 100000 --tag g2
OFR_F6P_GROUP=64 run --gallery 500000 --query-ids 100000 --tag g2_group64
run --gallery 250000 --query-ids 100000 --tag g4
run --gallery 125000 --query-ids 100000 --tag g8
OFR_F6P_GROUP=64 run --gallery 125000 --query-ids 100000 --tag g8_group64
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or sieve or shard" > gpurun_out/${T}_tests.txt 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.txt; exit $rc
