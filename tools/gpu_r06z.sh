# round 6: prefix wave pass in linear step order with the grouping rule: G = 1 (default, 16, 64), G = 8
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06z}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --engines 4,3 --tag g1
OFR_F6P_GROUP=16 run --engines 4 --tag g1_group16
OFR_F6P_GROUP=32 run --engines 4 --tag g1_group32
run --engines 4 --tag g1_again
run --engines 4 --gallery 125000 --query-ids 100000 --tag g8
run --engines 4 --gallery 500000 --query-ids 100000 --tag g2
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['engine'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1))"
