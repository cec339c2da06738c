#!/bin/bash
# A/B of the in-tree library against lib/exp/noslp.so on configs 2/4/5 (bench --no-extra) and the P=8 rank
# emulation of configs 3/5 (r06 no-SLP check).  GPU box: gpurun -- bash tools/ab_configs.sh
set -o pipefail
mkdir -p gpurun_out/abc
for r in 1 2; do for L in base noslp; do
  if [ $L = base ]; then LIB=$PWD/gpu_raytracer_amd/lib/librtamd.so; else LIB=$PWD/gpu_raytracer_amd/lib/exp/$L.so; fi
  for c in 2 4 5; do
    RT_LIB=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --config $c --steps 10 > gpurun_out/abc/${L}_c${c}_$r.json 2> gpurun_out/abc/${L}_c${c}_$r.err || exit 1
    echo "$L c$c $r $(python3 -c "import json;d=json.load(open('gpurun_out/abc/${L}_c${c}_$r.json'));print('trace',d['trace_ms'],'build',d['build_ms'],'value',d['value'],'crc',d['image_crc32'])")"
  done
  for c in 3 5; do
    RT_LIB=$LIB timeout -k 10 200 python tools/rank_emul.py config=$c frames=6 ranks=8 2>/dev/null | python3 tools/emul_line.py "$L c$c r$r" || exit 1
  done
done; done
