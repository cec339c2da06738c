#!/bin/bash
# Wide-stack depth A/B on the bench line (full frames, N=1): the library
# against variants built with tools/build_exp.sh stk16 "-DRT_WIDE_STACK=16" ...
# (RT_WIDE_STACK sets the 256-thread kernels' depth).  GPU box:
#   gpurun -- bash tools/ab_stack.sh   -> gpurun_out/abstk/
set -o pipefail
mkdir -p gpurun_out/abstk
for r in 1 2; do
  for L in base stk16 stk18 stk20 stk24; do
    if [ $L = base ]; then LIB=gpu_raytracer_amd/lib/librtamd.so; else LIB=gpu_raytracer_amd/lib/exp/$L.so; fi
    RT_LIB=$PWD/$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > gpurun_out/abstk/${L}_$r.json 2> gpurun_out/abstk/${L}_$r.err || exit 1
    echo "$L $r $(python3 -c "import json;d=json.load(open('gpurun_out/abstk/${L}_$r.json'));print(d['trace_ms'],d['value'],d['build_ms'],d['value_static_camera_best_case'])")"
  done
done
