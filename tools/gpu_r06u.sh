# round 6: the prefix tier's sample pass and sieve pass on one rank's shard (G = 1, 8; foreign queries at 8)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06u}
: > gpurun_out/${T}_probe.jsonl
timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 --tag g1 >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe1.log || { tail -20 gpurun_out/${T}_probe1.log; exit 1; }
timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4,3 --gallery 125000 --query-ids 100000 --tag g8 >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe8.log || { tail -20 gpurun_out/${T}_probe8.log; exit 1; }
timeout -k 10 200 python -u tools/probe_prefix_pass.py --engines 4 --gallery 125000 --tag g8own >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe8o.log || { tail -20 gpurun_out/${T}_probe8o.log; exit 1; }
cat gpurun_out/${T}_probe.jsonl
