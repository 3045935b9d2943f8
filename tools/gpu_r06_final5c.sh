# round-6 final tree: rocprofv3 stats + PMC of the headline launches only (no configs[1]/[3]/[4]/API side runs):
# the prefix pass, then the merge
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
A="--steps 4 --warmup 2 --small-batches= --stress= --config1 0 --config3 0 --config4 0 --api 0 --no-cpu"
bash tools/prof_search.sh "prefix_wave_kernel" $A || exit $?
mv gpurun_out/prof gpurun_out/prof_prefix5
bash tools/prof_search.sh "merge_kernel" $A || exit $?
mv gpurun_out/prof gpurun_out/prof_merge5
# keep gpurun_out under the 64 MiB merge limit: the per-dispatch trace only for the kernels of interest
for d in gpurun_out/prof_prefix5 gpurun_out/prof_merge5; do
  f=$d/kt/kt_kernel_trace.csv
  { head -1 $f; grep -E "prefix_wave_kernel|merge_kernel|project_q8w_kernel|sample_wave_kernel" $f; } > $f.sel && mv $f.sel $f
done
du -sh gpurun_out
