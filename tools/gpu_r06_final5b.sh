# round-6 final tree: smoke, the default bench line, rocprofv3 stats + PMC of the prefix pass
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=r06_final5
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
cut -c1-400 gpurun_out/${T}_bench.json
bash tools/prof_search.sh "prefix_wave_kernel" || exit $?
mv gpurun_out/prof gpurun_out/prof_prefix
