# round 6: one rank's share of the sharded step at the f6p operating point (trained W), G = 1/2/4/8
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06t}
: > gpurun_out/${T}_rank_share.jsonl
for G in 1 2 4 8; do
timeout -k 10 300 python -u tools/probe_rank_share.py --gpus $G >> gpurun_out/${T}_rank_share.jsonl 2> gpurun_out/${T}_rank_share_$G.log || { tail -20 gpurun_out/${T}_rank_share_$G.log; exit 1; }
tail -1 gpurun_out/${T}_rank_share.jsonl
done
