# Row sample (ofr_knn_f6_sampled, default) vs panel sample (OFR_SIEVE_SAMPLE=panels): the sieve GPU tests,
# then two alternating bench rounds, headline + configs[1] step.  One line per run in gpurun_out/r04rs/ab.txt.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04rs
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $R/tests/test_gpu_sieve.py > $O/tests.txt 2>&1
for rep in 1 2; do
  for mode in rows panels; do
    OFR_SIEVE_SAMPLE=$mode timeout -k 10 200 python3 $R/bench.py --steps 10 --no-cpu --stress= --small-batches= > $O/b_${mode}_$rep.json 2>> $O/err.txt
    python3 - $O/b_${mode}_$rep.json $mode >> $O/ab.txt <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = r["kernels_ms"]; c = r["config1"]
print(sys.argv[2], round(r["value"]), round(r["ms_per_step"], 3), round(r["roofline"]["launch_ms"], 3),
      round(r["roofline"]["phase1"]["sample_ms"], 3), round(k["knn_merge_rerank+certificate"], 3),
      r["sieve_kept_rows_per_query"]["mean"], r["sieve_kept_rows_per_query"]["max"], r["uncertified_after_each_tier"],
      round(c["queries_per_s"]), round(c["ms_per_step"], 3), c["uncertified_after_each_tier"], r["top1_identity_acc"])
PY
  done
done
echo done
