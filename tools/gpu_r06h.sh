# round 6: where the prefix pass's time goes (probe builds, tools/build_pp_probes.sh 0 1 2 4 6 7) and an
# isolated profile of the B = 4096 projection launch (tools/bench_proj.py --child at the bench shape)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
T=${TAG:-r06h}
: > gpurun_out/${T}_probe.jsonl
for L in in-tree 0 1 2 4 6 7; do
  if [ "$L" = "in-tree" ]; then unset OFR_LIB; else export OFR_LIB=tools/var/libpp_$L.so; fi
  timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 2 --tag pp$L >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || exit $?
done
unset OFR_LIB
cat gpurun_out/${T}_probe.jsonl
P="$R/tools/bench_proj.py --child --out /tmp/bproj --reps 20"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_proj/kt -o kt -- python3 $P > $R/gpurun_out/${T}_proj_kt.log 2>&1 || exit $?
K=project_q8w
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-include-regex $K --output-format csv -d $R/gpurun_out/${T}_proj/p1 -o p1 -- python3 $P > $R/gpurun_out/${T}_proj_p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/${T}_proj/p2 -o p2 -- python3 $P > $R/gpurun_out/${T}_proj_p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/${T}_proj/p3 -o p3 -- python3 $P > $R/gpurun_out/${T}_proj_p3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/${T}_proj/p4 -o p4 -- python3 $P > $R/gpurun_out/${T}_proj_p4.log 2>&1 || exit $?
echo prof ok
