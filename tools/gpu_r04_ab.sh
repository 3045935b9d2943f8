# Same-box A/B of the current library against a baseline build (tools/var/libocvf_base.so via OFR_LIB):
# the sieve GPU tests on the current library, then the bench (headline + configs[1]), two alternating
# rounds.  Usage: bash tools/gpu_r04_ab.sh <tag>; output under gpurun_out/ab_<tag>/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $R/tests/test_gpu_sieve.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_configs.py -k "sieve or projection or project or duplicate or row_sample or f6x2" > $O/tests.txt 2>&1
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export OFR_LIB=$R/tools/var/libocvf_base.so; else unset OFR_LIB; fi
    timeout -k 10 300 python3 $R/bench.py --steps 10 --no-cpu --stress= --small-batches= > $O/b_${v}_$rep.json 2>> $O/err.txt
    python3 - $O/b_${v}_$rep.json $v >> $O/ab.txt <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = r["config1"]
print(sys.argv[2], round(r["value"]), round(r["ms_per_step"], 3), round(r["roofline"]["launch_ms"], 3),
      r["uncertified_after_each_tier"], round(c["queries_per_s"]), round(c["ms_per_step"], 3))
PY
  done
done
unset OFR_LIB
cat $O/ab.txt
