# round 6: 128 x 32 wave steps (OFR_F6P_WAVE=8) with its grouping (>= 12 items per workgroup) at G = 1/2/4/8 shard sizes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06af}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
export OFR_F6P_WAVE=8
run --tag g1_w8
run --gallery 500000 --query-ids 100000 --tag g2_w8
OFR_F6P_GROUP=32 run --gallery 500000 --query-ids 100000 --tag g2_w8_q32
run --gallery 250000 --query-ids 100000 --tag g4_w8
OFR_F6P_GROUP=16 run --gallery 250000 --query-ids 100000 --tag g4_w8_q16
run --gallery 125000 --query-ids 100000 --tag g8_w8
OFR_F6P_GROUP=16 run --gallery 125000 --query-ids 100000 --tag g8_w8_q16
OFR_F6P_WAVE=4 run --gallery 500000 --query-ids 100000 --tag g2_w4
OFR_F6P_WAVE=4 run --gallery 250000 --query-ids 100000 --tag g4_w4
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['engine'], round(d['pass_ms_median'],3), round(d['kept_mean'],1), d['kept_max'])"
