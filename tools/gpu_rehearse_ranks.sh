#!/bin/bash
# Rehearsal of the multi-rank bench step on ONE GPU: gloo, every rank on device 0 (OFR_ONE_DEVICE=1).
# Validates the sharded path at the driver's rank counts (shard ranges, B/G query panels, the
# all-gathers, the global certificate); its times mean nothing.  Usage: tools/gpu_rehearse_ranks.sh 4 8
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for G in "$@"; do
  OFR_DIST_BACKEND=gloo OFR_ONE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $G \
      --master-addr 127.0.0.1 --master-port $((29600 + G)) bench.py --gpus $G --steps 2 --warmup 1 --no-cpu \
      --small-batches "" --stress "" --config1 0 > gpurun_out/rehearse_$G.json 2> gpurun_out/rehearse_$G.log || exit $?
  python -c "import json;r=json.loads(open('gpurun_out/rehearse_$G.json').read().strip().splitlines()[-1]);print($G, r['n_gpus'], r['uncertified_after_each_tier'], r['top1_identity_acc'], r['config']['parallelism'])"
done
