#!/bin/bash
# Probe builds of the library for tools/probe_prefix_pass.py: ofr_knn_q8.hip with -DOFR_PP_PROBE=N (bits:
# 1 no bucket flush, 2 no compares, 4 no MFMAs) linked with the other objects of the in-tree build, into
# tools/var/libpp_N.so.  Run here (CPU, hipcc cross-compiles) after `make` in csrc.
set -eu
cd "$(dirname "$0")/../opencv_facerecognizer_amd/csrc"
mkdir -p ../../tools/var
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-variable -Wno-unused-command-line-argument -munsafe-fp-atomics"
for n in "$@"; do
  /opt/rocm/bin/hipcc $FLAGS -DOFR_PP_PROBE=$n -c ofr_knn_q8.hip -o build/pp_$n.o &
done
wait
for n in "$@"; do
  objs=$(ls build/*.o | grep -v -E "build/(pp_[0-9]+|ofr_knn_q8)\.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/var/libpp_$n.so $objs build/pp_$n.o
done
ls -la ../../tools/var
