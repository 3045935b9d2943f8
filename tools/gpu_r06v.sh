# round 6: prefix wave pass at a G = 8 shard (125k rows, 7/8 foreign queries): hit path cost (probe bit 8) and grouping
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06v}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --tag g1
OFR_LIB=tools/var/libpp_8.so run --tag g1_nohits
run --gallery 125000 --query-ids 100000 --tag g8
OFR_LIB=tools/var/libpp_8.so run --gallery 125000 --query-ids 100000 --tag g8_nohits
for G in 32 16 8 4; do OFR_F6P_GROUP=$G run --gallery 125000 --query-ids 100000 --tag g8_group$G; done
for G in 32 16; do OFR_F6P_GROUP=$G run --tag g1_group$G; done
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1))"
