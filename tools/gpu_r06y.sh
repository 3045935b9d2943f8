# round 6: reproducibility of the 1M prefix pass after the grouping change (engines 4, 3)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06y}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --engines 4,3,4,3 --tag g1
OFR_F6P_GROUP=16 run --engines 4 --tag g1_group16
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['engine'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1))"
