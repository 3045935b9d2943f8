#!/bin/bash
# Probe builds of the library for the projection engine (tools/bench_proj.py lib=...): ofr_qproj.hip with
# -DOFR_PROJ_PROBE=N (bits: 1 no main-loop barriers, 2 no main-loop stage copies; results WRONG, timing only)
# linked with the other objects of the in-tree build, into tools/var/libproj_N.so.  Run here after `make`.
set -eu
cd "$(dirname "$0")/../opencv_facerecognizer_amd/csrc"
mkdir -p ../../tools/var
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-variable -Wno-unused-command-line-argument -munsafe-fp-atomics"
for n in "$@"; do
  /opt/rocm/bin/hipcc $FLAGS -DOFR_PROJ_PROBE=$n -c ofr_qproj.hip -o build/proj_$n.o &
done
wait
for n in "$@"; do
  objs=$(ls build/*.o | grep -v -E "build/(proj_[0-9]+|pp_[0-9]+|ofr_qproj)\.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/var/libproj_$n.so $objs build/proj_$n.o
done
ls -la ../../tools/var
