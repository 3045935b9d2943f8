#!/bin/bash
# fp6 probe variants timed, then one PMC pass for clock and MFMA busy per variant (gpurun_out/pclk).
cd /tmp && export TMPDIR=/tmp; R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/pclk
SHAPE16=1 timeout -k 10 200 ./tools/f6_probe 1000000 4096 9999 2 > gpurun_out/pclk/probe.log 2>&1 || exit $?
cat gpurun_out/pclk/probe.log
cd /tmp && SHAPE16=1 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $R/gpurun_out/pclk/p -o p --output-format csv -- $R/tools/f6_probe 1000000 4096 9999 1 > $R/gpurun_out/pclk/pmc.log 2>&1
