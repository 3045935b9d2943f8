# round 6: where the prefix_pass_kernel's time goes (probe builds) + the deferred-flush build, then its tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06c}
: > gpurun_out/${T}_probe.jsonl
for L in in-tree tools/var/libpp_base.so tools/var/libpp_1.so tools/var/libpp_2.so tools/var/libpp_4.so; do
  if [ "$L" = "in-tree" ]; then unset OFR_LIB; E=2,1; else export OFR_LIB=$L; E=2; fi
  timeout -k 10 240 python -u tools/probe_prefix_pass.py --engines $E --tag $L >> gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}_probe.log || exit $?
done
unset OFR_LIB
cat gpurun_out/${T}_probe.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -k "prefix or sieve or headline or shard or sharded or pipeline" > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_gpu_tests.txt
exit $rc
