# round 6: projection engine probe builds (timing only: 1 no main-loop barriers, 2 no stage copies, 3 neither)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r06al}
timeout -k 10 400 python -u tools/bench_proj.py --engines lib=opencv_facerecognizer_amd/libocvf_hip.so,lib=tools/var/libproj_1.so,lib=tools/var/libproj_2.so,lib=tools/var/libproj_3.so,lib=opencv_facerecognizer_amd/libocvf_hip.so > gpurun_out/${T}_proj.json 2> gpurun_out/${T}_proj.log
cat gpurun_out/${T}_proj.log | cut -c1-200
exit 0
