#!/bin/bash
# rocprofv3 counter passes for the training / LBP / chi-square kernels (run on the GPU box from the
# repo root): one kernel-trace pass, then one --pmc pass per counter group (no trace domains
# mixed with --pmc), each under its own time limit.  Summarise locally with
#   python tools/pmc_aux_summary.py <name>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_auxpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K="gemm_f64_kernel|gram_u8_kernel|elbp_hist_r1p8_kernel|chi2_tile_kernel"
run() {   # tag, tool args...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/kt -o kt -- python3 "$@" \
      > $O/$tag/kt.log 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$K" --output-format csv -d $O/$tag/p1 -o p1 -- python3 "$@" \
      > $O/$tag/p1.log 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" \
      --output-format csv -d $O/$tag/p2 -o p2 -- python3 "$@" > $O/$tag/p2.log 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $O/$tag/p3 -o p3 \
      -- python3 "$@" > $O/$tag/p3.log 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $O/$tag/p4 -o p4 \
      -- python3 "$@" > $O/$tag/p4.log 2>&1 || return $?
}
mkdir -p $O/gemm $O/lbp
run gemm $R/tools/bench_gemm.py || { echo "gemm passes failed rc=$?"; exit 1; }
run lbp $R/tools/bench_lbp_chi2.py --cpu-seconds 0.5 || { echo "lbp passes failed rc=$?"; exit 1; }
echo done
