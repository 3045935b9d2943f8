#!/bin/bash
# Probe builds of the library with merge_kernel's compile-time probe bits (OFR_MERGE_PROBE_V, see
# csrc/ofr_knn_q8.hip): tools/mprobe/libocvf_hip_v<V>.so, loaded by tools/probe_merge.py through
# OFR_LIB.  Needs the library's other objects built (make -C opencv_facerecognizer_amd/csrc).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/opencv_facerecognizer_amd/csrc
mkdir -p $R/tools/mprobe
for V in ${@:-1 2 4 7}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -DOFR_MERGE_PROBE_V=$V \
      -c $C/ofr_knn_q8.hip -o $R/tools/mprobe/ofr_knn_q8_v$V.o
  objs=$(ls $C/build/*.o | grep -v ofr_knn_q8.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/mprobe/libocvf_hip_v$V.so $objs \
      $R/tools/mprobe/ofr_knn_q8_v$V.o
  rm $R/tools/mprobe/ofr_knn_q8_v$V.o
done
