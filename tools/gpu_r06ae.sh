# round 6: prefix wave pass shapes: 64 rows x 64 queries per wave step (default) vs 128 x 32 (OFR_F6P_WAVE=8); tests under 8
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ae}
: > gpurun_out/${T}_probe.jsonl
run() { timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 "$@" >> gpurun_out/${T}_probe.jsonl 2>> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }; }
for r in 1 2; do
run --tag g1_w4
OFR_F6P_WAVE=8 run --tag g1_w8
done
run --gallery 125000 --query-ids 100000 --tag g8_w4
OFR_F6P_WAVE=8 run --gallery 125000 --query-ids 100000 --tag g8_w8
for q in 16 32; do OFR_F6P_WAVE=8 OFR_F6P_GROUP=$q run --tag g1_w8_q$q; done
cat gpurun_out/${T}_probe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['engine'], round(d['pass_ms_median'],3), round(d['kept_mean'],1), d['kept_max'])"
OFR_F6P_WAVE=8 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or sieve or headline" > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
