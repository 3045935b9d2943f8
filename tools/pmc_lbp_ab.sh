#!/bin/bash
# PMC counters of the LBP histogram kernels, the fp64 r1p8 kernel (OFR_LBP_EXACT64=1) beside the fast one
# (round 5: the fast kernel and its OFR_LBP_EXACT64 switch were measured and not shipped -- DESIGN.md §8;
# on the shipped library both passes time the same r1p8 kernel)
# (run on the GPU box from the repo root; one --pmc pass per group, no trace domains)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc_lbp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  export OFR_LBP_EXACT64=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
      SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU --kernel-include-regex "elbp_hist" \
      --output-format csv -d $O/v$v -o p1 -- python3 $R/tools/bench_lbp_chi2.py --cpu-seconds 0.1 --reps 1 \
      > $O/v$v.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, os
O = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "gpurun_out/pmc_lbp")
for v in ("1", "0"):
    f = glob.glob(f"{O}/v{v}/**/*counter_collection.csv", recursive=True)
    acc = {}
    for fn in f:
        for r in csv.DictReader(open(fn)):
            if "elbp" not in r["Kernel_Name"]:
                continue
            k = (r["Kernel_Name"][:40], r["Counter_Name"])
            acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"])
    print("OFR_LBP_EXACT64=" + v, {k[1]: v2 for k, v2 in sorted(acc.items())}, sorted({k[0] for k in acc}))
PY
