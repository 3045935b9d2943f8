# A/B of the sieve threshold: sample stride (OFR_SIEVE_STRIDE) x threshold rank (OFR_SIEVE_RANK), two
# alternating rounds, headline + configs[1] step.  One line per run in gpurun_out/r04sr/ab.txt.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04sr
mkdir -p $O
for rep in 1 2; do
  for cfg in ${CFGS:-64:16 128:16 256:16 64:12}; do
    st=${cfg%:*}; rk=${cfg#*:}
    OFR_SIEVE_STRIDE=$st OFR_SIEVE_RANK=$rk timeout -k 10 200 python3 $R/bench.py --steps 10 --no-cpu --stress= --small-batches= > $O/b_${st}_${rk}_$rep.json 2>> $O/err.txt
    python3 - $O/b_${st}_${rk}_$rep.json $st $rk >> $O/ab.txt <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = r["kernels_ms"]; c = r["config1"]
print(sys.argv[2], sys.argv[3], round(r["value"]), round(r["ms_per_step"], 3), round(r["roofline"]["launch_ms"], 3),
      round(r["roofline"]["phase1"]["sample_ms"], 3), round(k["knn_merge_rerank+certificate"], 3),
      r["sieve_kept_rows_per_query"]["mean"], r["sieve_kept_rows_per_query"]["max"], r["uncertified_after_each_tier"],
      round(c["queries_per_s"]), round(c["ms_per_step"], 3), c["uncertified_after_each_tier"], r["top1_identity_acc"])
PY
  done
done
echo done
