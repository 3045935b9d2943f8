# round 6: prefix_wave_kernel at 2 vs 3 workgroups per CU (168 VGPRs, 13 spills)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06q}
timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 4:2,4:3,4:2,4:3 --tag in-tree > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || { tail -20 gpurun_out/${T}_probe.log; exit 1; }
cat gpurun_out/${T}_probe.jsonl
