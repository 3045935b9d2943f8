# round 6: prefix wave pass with 2 query steps in flight (default) vs 1 (OFR_F6P_PREFETCH=1); tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ac}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
for r in 1 2; do
run --tag g1_pf2
OFR_F6P_PREFETCH=1 run --tag g1_pf1
done
run --gallery 125000 --query-ids 100000 --tag g8_pf2
OFR_F6P_PREFETCH=1 run --gallery 125000 --query-ids 100000 --tag g8_pf1
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['engine'], round(d['pass_ms_median'],3), round(d['sample_ms_median'],3), round(d['kept_mean'],1), d['kept_max'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or sieve" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
