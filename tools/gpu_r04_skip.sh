# (1) the sieve + sharded-training GPU tests and the two-slice pass probe on the current library;
# (2) A/B of the wide engine without the clamped tail copies (current) against the previous build
# (tools/var/libocvf_preskip.so via OFR_LIB), two alternating rounds.  Output under gpurun_out/r04sk/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04sk
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $R/tests/test_gpu_sieve.py $R/tests/test_gpu_configs.py -k "sieve or sharded_training or regimes or duplicate" > $O/tests.txt 2>&1
timeout -k 10 400 python3 $R/tools/probe_f6x2_pass.py > $O/f6x2_probe.jsonl 2> $O/f6x2_probe.err
for rep in 1 2; do
  for v in skip preskip; do
    if [ $v = preskip ]; then export OFR_LIB=$R/tools/var/libocvf_preskip.so; else unset OFR_LIB; fi
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
echo done
