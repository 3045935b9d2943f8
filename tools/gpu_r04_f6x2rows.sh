# Two-slice tier with the row sample (default) vs the panel sample (OFR_SIEVE_SAMPLE=panels): sieve GPU
# tests, then the stress runs (sigma 96, 192), alternating.  Output under gpurun_out/r04x2r/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04x2r
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $R/tests/test_gpu_sieve.py > $O/tests.txt 2>&1
for rep in 1 2; do
  for mode in rows panels; do
    OFR_SIEVE_SAMPLE=$mode timeout -k 10 300 python3 $R/bench.py --steps 5 --no-cpu --stress=96,192 --small-batches= > $O/b_${mode}_$rep.json 2>> $O/err.txt
  done
done
echo done
