# round 6: prefix_wave_kernel<8, 2> probe builds at 1M / B = 4,096: bit 2 no compares, bit 8 no hit path
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06aj}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
run --tag in-tree
OFR_LIB=tools/var/libpp_8.so run --tag no_hits
OFR_LIB=tools/var/libpp_2.so run --tag no_compares
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['pass_ms_median'],3), round(d['kept_mean'],1))"
