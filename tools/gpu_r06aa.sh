# round 6: prefix wave pass, steps per work item (OFR_F6P_GROUP) swept at G = 1/2/4/8 shard sizes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06aa}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
for q in 4 8 16; do OFR_F6P_GROUP=$q run --tag g1_q$q; done
for q in 8 16 32; do OFR_F6P_GROUP=$q run --gallery 500000 --query-ids 100000 --tag g2_q$q; done
for q in 4 8 16; do OFR_F6P_GROUP=$q run --gallery 250000 --query-ids 100000 --tag g4_q$q; done
for q in 2 4 8; do OFR_F6P_GROUP=$q run --gallery 125000 --query-ids 100000 --tag g8_q$q; done
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['engine'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1))"
