#!/bin/bash
# build-time A/B of library variants (tools/build_times.py per library, alternating)
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
for L in "$@"; do
  RT_LIB=$PWD/$L timeout -k 10 120 python -u tools/build_times.py 1000000 30 2>&1 | grep -v amdgpu.ids | tail -1
done
done
