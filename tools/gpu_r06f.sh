# round 6: the prefix pass engines A/B on one box -- alone (probe) and in the bench step, alternating
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06f}
timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 2,1,2,1 --tag in-tree > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || exit $?
cat gpurun_out/${T}_probe.jsonl
for e in 2 1 2 1; do
  OFR_F6P_ENGINE=$e timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --stress= --small-batches= --no-cpu --config1 0 --config3 0 --config4 0 --api 0 > gpurun_out/${T}_bench_e$e.json 2> gpurun_out/${T}_bench_e$e.log || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench_e$e.json').read());print('engine $e', round(d['value']), d['ms_per_step'], d['kernels_ms'], d['roofline']['launch_ms'], d['uncertified_after_each_tier'])"
done
