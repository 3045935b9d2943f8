# round-4 investigation: configs[1]-shaped kernel trace, tile-group A/B of the wide sieve pass, and
# the L2<->fabric traffic of gg = 2 / 4 (one PMC pass each).  Run from the repo root on the GPU box.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu --stress= --config1 0 --small-batches="
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c1 -o c1 -- python3 $R/bench.py --gallery 100000 --steps 10 $Q > $O/c1.log 2>&1
for g in 2 4 2 4; do
  OFR_F6W_GROUP=$g timeout -k 10 200 python3 $R/bench.py --steps 10 $Q > $O/gg$g.json 2>> $O/gg.err
  python3 -c "import json,sys; r=json.loads(open('$O/gg$g.json').read().strip().splitlines()[-1]); print($g, r['roofline']['launch_ms'], r['ms_per_step'], r['value'])" >> $O/gg_ab.txt
done
for g in 2 4; do
  OFR_F6W_GROUP=$g timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tile_kernel_f6w --output-format csv -d $O/pf$g -o pf -- python3 $R/bench.py --steps 2 --warmup 1 $Q > $O/pf$g.log 2>&1
  OFR_F6W_GROUP=$g timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-include-regex tile_kernel_f6w --output-format csv -d $O/pw$g -o pw -- python3 $R/bench.py --steps 2 --warmup 1 $Q > $O/pw$g.log 2>&1
done
echo done
