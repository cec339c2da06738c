#!/bin/bash
# Bench-line A/B of library variants (N=1, no CPU baseline, no extras):
# alternating rounds, one bench.py process per library (RT_LIB).  Variants
# come from tools/build_exp.sh (gpu_raytracer_amd/lib/exp/<name>.so); "base"
# is the in-tree library.  GPU box:
#   gpurun -- bash tools/ab_bench_libs.sh ROUNDS name [name ...]   -> gpurun_out/abl/
set -o pipefail
rounds=$1; shift
mkdir -p gpurun_out/abl
for r in $(seq 1 $rounds); do
  for L in "$@"; do
    if [ $L = base ]; then LIB=gpu_raytracer_amd/lib/librtamd.so; else LIB=gpu_raytracer_amd/lib/exp/$L.so; fi
    RT_LIB=$PWD/$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > gpurun_out/abl/${L}_$r.json 2> gpurun_out/abl/${L}_$r.err || exit 1
    echo "$L $r $(python3 -c "import json;d=json.load(open('gpurun_out/abl/${L}_$r.json'));print('trace_ms',d['trace_ms'],'value',d['value'],'static',d['value_static_camera_best_case'],'cold',d['value_cold'])")"
  done
done
