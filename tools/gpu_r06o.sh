# round 6: PMC of the folded prefix pass (in-tree) against its no-hit-path probe (bit 8) and no-flush probe (bit 1)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
T=${TAG:-r06o}
cd /tmp && export TMPDIR=/tmp
P="$R/tools/probe_prefix_pass.py --engines 3 --reps 3"
for L in in-tree 8 1; do
  if [ "$L" = "in-tree" ]; then unset OFR_LIB; else export OFR_LIB=$R/tools/var/libpp_$L.so; fi
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex prefix_pass --output-format csv -d $R/gpurun_out/${T}_$L/p1 -o p1 -- python3 $P > $R/gpurun_out/${T}_${L}_p1.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex prefix_pass --output-format csv -d $R/gpurun_out/${T}_$L/p2 -o p2 -- python3 $P > $R/gpurun_out/${T}_${L}_p2.log 2>&1 || echo "p2 $L failed"
done
echo done
