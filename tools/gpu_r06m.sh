# round 6: where the folded prefix pass's (engine 3) time goes -- probe builds (tools/build_pp_probes.sh 1 2 6 8)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06m}
: > gpurun_out/${T}_probe.jsonl
for L in in-tree 1 2 6 8 in-tree; do
  if [ "$L" = "in-tree" ]; then unset OFR_LIB; else export OFR_LIB=tools/var/libpp_$L.so; fi
  timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines 3 --tag pp$L >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || exit $?
done
cat gpurun_out/${T}_probe.jsonl
