#!/bin/bash
# GPU call: the headline bench on one GPU (short), then the 2-rank rehearsal of the sharded step
# on the same GPU (gloo, both ranks on device 0: exercises the multi-rank code path; its times mean
# nothing).  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
T=${1:-r02_check}
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu --small-batches "" --stress "" --config1 0 \
    > gpurun_out/${T}_bench1.json 2> gpurun_out/${T}_bench1.log || exit $?
cut -c1-700 gpurun_out/${T}_bench1.json
OFR_DIST_BACKEND=gloo OFR_ONE_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --small-batches "" \
    --stress "" --config1 0 > gpurun_out/${T}_bench2r.json 2> gpurun_out/${T}_bench2r.log || exit $?
cut -c1-700 gpurun_out/${T}_bench2r.json
