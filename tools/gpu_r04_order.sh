# A/B of the wide sieve pass's tile order: tile-group width (OFR_F6W_GROUP) x serpentine query order
# (OFR_F6W_SERP), two alternating rounds, then one FETCH_SIZE pass per variant.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ord
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
Q="--no-cpu --stress= --config1 0 --small-batches="
for rep in 1 2; do
  for cfg in ${CFGS:-2:0 2:1 4:0 4:1}; do
    g=${cfg%:*}; sp=${cfg#*:}
    OFR_F6W_GROUP=$g OFR_F6W_SERP=$sp timeout -k 10 200 python3 $R/bench.py --steps 10 $Q > $O/b_${g}_${sp}_$rep.json 2>> $O/err.txt
    python3 -c "import json; r=json.loads(open('$O/b_${g}_${sp}_$rep.json').read().strip().splitlines()[-1]); print($g, $sp, round(r['value']), round(r['roofline']['launch_ms'],3), round(r['ms_per_step'],3))" >> $O/ab.txt
  done
done
for cfg in ${CFGS:-2:0 2:1 4:0 4:1}; do
  g=${cfg%:*}; sp=${cfg#*:}
  OFR_F6W_GROUP=$g OFR_F6W_SERP=$sp timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tile_kernel_f6w --output-format csv -d $O/pf_${g}_${sp} -o pf -- python3 $R/bench.py --steps 2 --warmup 1 $Q > $O/pf_${g}_${sp}.log 2>&1
  python3 -c "
import csv,glob
rows=[r for r in csv.DictReader(open(glob.glob('$O/pf_${g}_${sp}/*counter_collection.csv')[0])) if r['Counter_Name']=='FETCH_SIZE']
v=[float(r['Counter_Value']) for r in rows]
print('fetch', $g, $sp, len(v), 2*sum(v)/len(v)/1e6, 'GB per launch (FETCH_SIZE x2, KB units)')" >> $O/ab.txt
done
echo done
