# rocprofv3 evidence for the search pass (run on the GPU box from the repo root):
#   bash tools/prof_search.sh [kernel-regex] [bench args...]
# kernel trace + stats, then one PMC pass per counter group (no trace domains mixed with --pmc).
set -e
R=$GRAFT_REPO_ROOT
K=${1:-tile_kernel_f6|sieve_threshold}
shift || true
ARGS=${*:---steps 2 --warmup 1 --small-batches= --stress= --config1 0 --no-cpu}
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o kt -- python3 $B > $R/gpurun_out/prof/kt.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex $K --output-format csv -d $R/gpurun_out/prof/p1 -o p1 -- python3 $B > $R/gpurun_out/prof/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex $K --output-format csv -d $R/gpurun_out/prof/p2 -o p2 -- python3 $B > $R/gpurun_out/prof/p2.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/prof/p3 -o p3 -- python3 $B > $R/gpurun_out/prof/p3.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/prof/p4 -o p4 -- python3 $B > $R/gpurun_out/prof/p4.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/prof/p5 -o p5 -- python3 $B > $R/gpurun_out/prof/p5.log 2>&1
echo done
