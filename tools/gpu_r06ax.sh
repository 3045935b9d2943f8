# round 6: placement of the register-staged projection stores (tools/var/libprojv_<row0>_<stride>.so) vs LDS-DMA
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06ax}
OFR_PROJ_STAGE=reg timeout -k 10 400 python -u tools/bench_proj.py --engines dma,reg,lib=tools/var/libprojv_4_2.so,lib=tools/var/libprojv_8_1.so,lib=tools/var/libprojv_14_1.so,dma > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.log || { tail -30 gpurun_out/${T}_proj.log; cat gpurun_out/${T}_proj.json; exit 1; }
cat gpurun_out/${T}_proj.json
