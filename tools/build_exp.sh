#!/bin/bash
# Build timing experiments: compile librtamd variants with -D flags into
# gpu_raytracer_amd/lib/exp/<name>.so (never shipped), then time the build
# stages of each with tools/build_times.py (RT_LIB selects the library).
# usage (container): tools/build_exp.sh name "-DFLAG1 -DFLAG2" ...   (pairs)
set -e
cd "$(dirname "$0")/../gpu_raytracer_amd"
mkdir -p lib/exp build/exp
FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -std=c++17 -Wno-unused-function"
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  for f in build_kernels sort_kernels trace_kernels; do
    /opt/rocm/bin/hipcc $FLAGS $defs -c csrc/$f.hip -o build/exp/${name}_$f.o &
  done
  /opt/rocm/bin/hipcc $FLAGS $defs -x hip -c csrc/rt_abi.cpp -o build/exp/${name}_rt_abi.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/exp/$name.so build/exp/${name}_build_kernels.o \
    build/exp/${name}_sort_kernels.o build/exp/${name}_trace_kernels.o build/exp/${name}_rt_abi.o build/scene_io.o
  echo "built lib/exp/$name.so"
done
