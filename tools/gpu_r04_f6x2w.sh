# The two-slice tier on the wide engine: sieve / parity / pipeline GPU tests, then the stress runs
# (sigma 96, 192: every query goes fp6 -> f6x2) with the wide engine (default) and the 8-wave one
# (OFR_F6_SHAPE=16, both tiers), alternating.  Output under gpurun_out/r04x2/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04x2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $R/tests/test_gpu_sieve.py $R/tests/test_gpu_pipeline.py > $O/tests.txt 2>&1
for rep in 1 2; do
  for shape in 384 16; do
    OFR_F6_SHAPE=$shape timeout -k 10 300 python3 $R/bench.py --steps 5 --no-cpu --stress=96,192 --small-batches= > $O/b_${shape}_$rep.json 2>> $O/err.txt
  done
done
echo done
