# round 6: the prefix pass's hit path (probe bit 8) and its PMC (in-tree build)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
T=${TAG:-r06i}
: > gpurun_out/${T}_probe.jsonl
for L in in-tree 0 8 in-tree 8; do
  if [ "$L" = "in-tree" ]; then unset OFR_LIB; else export OFR_LIB=tools/var/libpp_$L.so; fi
  timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 2 --tag pp$L >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || exit $?
done
unset OFR_LIB
cat gpurun_out/${T}_probe.jsonl
P="$R/tools/probe_prefix_pass.py --engines 2 --reps 3"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-include-regex prefix_pass --output-format csv -d $R/gpurun_out/${T}_pp/p1 -o p1 -- python3 $P > $R/gpurun_out/${T}_pp_p1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex prefix_pass --output-format csv -d $R/gpurun_out/${T}_pp/p2 -o p2 -- python3 $P > $R/gpurun_out/${T}_pp_p2.log 2>&1 || echo "p2 failed $?"
echo prof ok
