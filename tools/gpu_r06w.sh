# round 6: prefix wave pass with per-workgroup rotated step order: G = 1 and a G = 8 shard, grouping
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06w}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --tag g1
run --gallery 125000 --query-ids 100000 --tag g8
for G in 16 8; do OFR_F6P_GROUP=$G run --gallery 125000 --query-ids 100000 --tag g8_group$G; done
for G in 16 8; do OFR_F6P_GROUP=$G run --tag g1_group$G; done
run --gallery 250000 --query-ids 100000 --tag g4
OFR_F6P_GROUP=8 run --gallery 250000 --query-ids 100000 --tag g4_group8
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1))"
